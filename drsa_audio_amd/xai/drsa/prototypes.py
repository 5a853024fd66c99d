"""Prototype search, drop-in for ``cxai.xai.drsa.prototypes.get_prototypes_ts``.

``prototypes.py:14-130``: shuffle the class's instances with ``torch.randperm`` (seeded
generator), cut them into subsets of ``n``, extract every-location activation/context vectors
per subset (``preprocess_data`` inference branch), score each subset with the DRSA objective of
U, and return the best subset's vectors, names and slice start points.

Here the data batch is passed in (the reference loads it from GTZAN folders with
``get_songs_drsa``, dataset I/O that is out of scope).  The LRP capture runs once for all N
instances on the HIP engine (results do not depend on the subset split) and each subset's
objective is one ``drsa_amd_drsa_objective`` call on a slice of the device vectors.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn as nn

from ...utils.constants import AUDIO_PARAMS
from ...utils.sound import round_down
from .drsa import DrsaWorkspace, drsa_objective
from .preprocessing import preprocess_data


def subset_objectives(act_vecs: torch.Tensor, ctx_vecs: torch.Tensor, U: torch.Tensor, num_concepts: int,
                      n: int) -> torch.Tensor:
    """DRSA objective of every block of n instances: act/ctx [N, HW, d] -> [N // n] (device)."""
    Nn, HW, d = act_vecs.shape
    ws = DrsaWorkspace(n * HW, d, num_concepts, act_vecs.device)
    out = []
    for i in range(Nn // n):
        a = act_vecs[i * n:(i + 1) * n].reshape(-1, d).contiguous()
        c = ctx_vecs[i * n:(i + 1) * n].reshape(-1, d).contiguous()
        out.append(drsa_objective(a, c, U, num_concepts, ws))
    return torch.stack(out) if out else torch.empty(0, device=act_vecs.device)


def get_prototypes_ts(model: nn.Module, layer_idx: int, U: torch.Tensor, composite, data_batch: torch.Tensor,
                      class_idx: int, loaded_samples: Optional[Sequence[str]] = None, case: str = "gtzan",
                      num_concepts: int = 4, n: int = 10, N: Optional[int] = None, seed: int = 42,
                      device=None) -> Tuple[torch.Tensor, torch.Tensor, List[str], Optional[torch.Tensor]]:
    """(prototype act vecs [n*HW, d], ctx vecs, songs, startpoints) of the best subset."""
    dev = torch.device(device) if device is not None else data_batch.device
    B = data_batch.size(0)
    N = N if N else B
    gen = torch.Generator().manual_seed(seed)
    perm = torch.randperm(B, generator=gen)
    startpoints = None
    if case == "gtzan":
        p = AUDIO_PARAMS["gtzan"]
        hop = round_down((29 - p["slice_length"]) / (p["num_chunks"] - 1), 1)
        startpoints = (torch.arange(p["num_chunks"]) * hop).repeat(B // p["num_chunks"])[perm][:N]
    x = data_batch[perm][:N].to(dev)
    names = list(loaded_samples) if loaded_samples is not None else [str(i) for i in range(B)]
    names = [names[i] for i in perm[:N]]
    A, C = preprocess_data(model, x, composite, layer_idx, class_idx, num_locations=None, device=dev)
    U = U.to(dev, torch.float32).contiguous()
    objs = subset_objectives(A, C, U, num_concepts, n)
    best = int(torch.argmax(objs).item()) if objs.numel() else 0
    # the reference keeps the first maximum over strictly-greater updates starting at 0
    if objs.numel() and float(objs.max()) <= 0:
        raise ValueError("no subset has a positive DRSA objective")
    a = A[best * n:(best + 1) * n].reshape(-1, A.size(-1)).clone()
    c = C[best * n:(best + 1) * n].reshape(-1, C.size(-1)).clone()
    sp = startpoints[best * n:(best + 1) * n] if startpoints is not None else None
    return a, c, names[best * n:(best + 1) * n], sp
