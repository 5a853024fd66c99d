"""DRSA dataset files, drop-in for ``cxai.xai.drsa.cluster.getdrsadata``.

* ``save_data``                — getdrsadata.py:26-44: ``{output_path}/{case}/{model}/{class}/
                                 dataset_layer{L}.pkl`` = pickle of ``list(zip(A, C))``
* ``load_and_normalize_data``  — getdrsadata.py:47-59: load that file, move to the device,
                                 ``normalize_vectors`` on A and C separately (HIP kernel)

These read and write the caller's own dataset files (the reference's format, so datasets made
by either side load in the other).  ``load_and_normalize_data`` reads the file with a restricted
unpickler that admits only numpy arrays / torch tensors (``utils/safe_pickle.py``).
"""
from __future__ import annotations

import os
import pickle

import numpy as np
import torch

from ....utils import safe_pickle
from ..preprocessing import normalize_vectors


def save_data(activation_vectors, context_vectors, layer=None, sample_class=None, case="gtzan", model="bn",
              output_path=None) -> str:
    assert type(layer) == int, "layer has to be defined and of type int"
    assert type(sample_class) == str, "sample_class has to be defined and of type str"
    assert output_path is not None, "please provide an output path to save the data"
    a = activation_vectors.detach().cpu().numpy() if torch.is_tensor(activation_vectors) else activation_vectors
    c = context_vectors.detach().cpu().numpy() if torch.is_tensor(context_vectors) else context_vectors
    path = os.path.join(output_path, f"{case}/{model}/{sample_class}")
    os.makedirs(path, exist_ok=True)
    filepath = os.path.join(path, f"dataset_layer{layer}.pkl")
    with open(filepath, "wb") as fh:
        pickle.dump(list(zip(a, c)), fh)
    return filepath


def load_and_normalize_data(filepath, device):
    with open(filepath, "rb") as fh:
        dataset = safe_pickle.load(fh)
    a, c = zip(*dataset)
    a = torch.tensor(np.array([np.asarray(v.cpu() if torch.is_tensor(v) else v) for v in a]), device=device,
                     dtype=torch.float32).contiguous()
    c = torch.tensor(np.array([np.asarray(v.cpu() if torch.is_tensor(v) else v) for v in c]), device=device,
                     dtype=torch.float32).contiguous()
    return normalize_vectors(a), normalize_vectors(c)
