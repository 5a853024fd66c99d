"""Run selection and artefact loading of the reference, host-side.

* ``get_run_stats`` / ``get_best_run``  — cxai/utils/evaluation.py:108-141 (pick the DRSA run
  with the highest final objective among ``run{r}/train_stats.csv``)
* ``load_projection_matrix``            — cxai/xai/pixelflipping/cpf.py:184-189 (U of the best
  run: ``{path}/{genre}/layer{j}/run{r}/projection_matrix.pkl``)
* ``save_checkpoint`` / ``load_checkpoint_state`` — the CNN checkpoint dict of
  cxai/model/train.py:175-188 (``best_model_{epoch}.pth`` with ``model_state_dict``)

These read and write the caller's own files (the formats ``drsa.main`` / ``SubspaceOptimizer``
write here and in the reference).  Checkpoints are loaded with ``weights_only=True``; the
reference's RNG-state entries are admitted through an explicit allowlist of numpy types.
``projection_matrix.pkl`` is read with a restricted unpickler that admits only arrays
(``utils/safe_pickle.py``).
"""
from __future__ import annotations

import os
import random
from typing import List, Tuple

import numpy as np
import pandas as pd
import torch

from . import safe_pickle


def get_run_stats(path: str) -> Tuple[float, List[float], List[float]]:
    """(final loss, final concept relevances of columns R*, all losses) of one train_stats.csv."""
    stats = pd.read_csv(path)
    final_loss = list(stats["loss"])[-1]
    concept_relevances = [list(stats[k])[-1] for k in stats.keys() if k.startswith("R")]
    return final_loss, concept_relevances, list(stats["loss"])


def get_best_run(path: str):
    """(best_run, best_loss, concept_relevances, path_to_best_run, train_losses) over the
    ``run{r}`` directories of ``path`` (highest final objective wins, first on ties)."""
    best_loss, best_run, best_path, best_rel, best_losses = 0, None, None, None, None
    for d in sorted(x for x in os.listdir(path) if not x.startswith(".")):
        run = int(d[-1])
        loss, rel, losses = get_run_stats(os.path.join(path, d, "train_stats.csv"))
        if loss > best_loss:
            best_loss, best_run, best_path, best_rel, best_losses = loss, run, os.path.join(path, d), rel, losses
    return best_run, best_loss, best_rel, best_path, best_losses


def load_projection_matrix(genre: str, layer_idx: int, path: str, device=torch.device("cpu")) -> torch.Tensor:
    _, _, _, best, _ = get_best_run(os.path.join(path, f"{genre}/layer{layer_idx}"))
    with open(os.path.join(best, "projection_matrix.pkl"), "rb") as fh:
        U = safe_pickle.load(fh)
    return torch.tensor(U, device=device)


def save_checkpoint(model_path: str, model_state, opt_state, epoch: int) -> str:
    path = os.path.join(model_path, "best_model_%s.pth" % epoch)
    torch.save({"model_state_dict": model_state, "opt_state_dict": opt_state,
                "random_rng_state": random.getstate(), "torch_rng_state": torch.get_rng_state(),
                "numpy_rng_state": np.random.get_state()}, path)
    return path


def _numpy_safe_globals():
    out = [np.ndarray, np.dtype, type(np.dtype(np.uint32))]
    try:
        from numpy.core.multiarray import _reconstruct
        out.append(_reconstruct)
    except ImportError:   # pragma: no cover
        pass
    try:
        from numpy._core.multiarray import _reconstruct as r2
        out.append(r2)
    except ImportError:   # pragma: no cover
        pass
    return out


def load_checkpoint_state(path: str, map_location="cpu") -> dict:
    """The ``model_state_dict`` of a reference-format checkpoint (weights_only load)."""
    with torch.serialization.safe_globals(_numpy_safe_globals()):
        ck = torch.load(path, map_location=map_location, weights_only=True)
    return ck["model_state_dict"] if isinstance(ck, dict) and "model_state_dict" in ck else ck
