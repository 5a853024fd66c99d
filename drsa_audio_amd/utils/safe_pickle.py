"""Restricted unpickling for the reference's array pickles (no code execution from the file).

The reference stores DRSA artefacts as plain pickles: ``projection_matrix.pkl`` (a float32 numpy
d x d, cxai/xai/drsa/drsa.py:165-168) and ``dataset_layer{L}.pkl`` (a list of (a, c) pairs of
rows, cxai/xai/drsa/cluster/getdrsadata.py:26-44; numpy rows here, torch tensors when the
reference wrote them).  ``load`` admits exactly the globals those need: numpy array / dtype
reconstruction, and torch's tensor rebuild with its storages read through ``torch.load(...,
weights_only=True)``.  Anything else (os.system, builtins.eval, arbitrary classes) raises
``pickle.UnpicklingError``.
"""
from __future__ import annotations

import io
import pickle
from typing import Any, BinaryIO

import numpy as np

_NUMPY = {("numpy", "ndarray"), ("numpy", "dtype"), ("numpy.core.multiarray", "_reconstruct"),
          ("numpy._core.multiarray", "_reconstruct"), ("numpy.core.multiarray", "scalar"),
          ("numpy._core.multiarray", "scalar"), ("numpy", "float32"), ("numpy", "float64"), ("numpy", "int64")}
_TORCH = {("torch._utils", "_rebuild_tensor_v2"), ("torch._utils", "_rebuild_tensor"), ("collections", "OrderedDict"),
          ("torch", "FloatStorage"), ("torch", "DoubleStorage"), ("torch", "HalfStorage"), ("torch", "BFloat16Storage"),
          ("torch", "LongStorage"), ("torch", "IntStorage"), ("torch.storage", "UntypedStorage"),
          ("torch", "float32"), ("torch", "float64")}


def _storage_from_bytes(b: bytes):
    """torch.storage._load_from_bytes, but through the weights_only loader."""
    import torch
    return torch.load(io.BytesIO(b), weights_only=True)


class ArrayUnpickler(pickle.Unpickler):
    def find_class(self, module: str, name: str) -> Any:
        if module == "numpy.dtypes" and name.endswith("DType"):
            return getattr(np.dtypes, name)
        if (module, name) == ("torch.storage", "_load_from_bytes"):
            return _storage_from_bytes
        if (module, name) in _NUMPY or (module, name) in _TORCH:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"refusing to unpickle {module}.{name}: only numpy arrays and torch tensors "
                                     f"are admitted (drsa_audio_amd.utils.safe_pickle)")


def load(fh: BinaryIO) -> Any:
    return ArrayUnpickler(fh).load()
