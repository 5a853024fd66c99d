"""ORACLE -- test infrastructure only (imported by tests/, never by drsa_audio_amd).

Loop-for-loop CPU restatement of the reference's concept-flipping evaluation
(cxai/xai/pixelflipping/cpf.py:87-395), with the defect resolutions documented in
drsa_audio_amd/xai/pixelflipping/cpf.py (D14 batch indexing reproduced, D15 intended return
values, D16 frob with the current K):

* interclass_concept_flipping  cpf.py:87-181   one HeatmapGenerator per (projection genre i,
                                                attributed genre j) on class batch i (D14), flipped
                                                over the whole batch, class means per row
* cf_random_subspace           cpf.py:192-233  ortho_group.rvs(dim), compounding permutations, the
                                                last permutation's heatmaps
* perform_cf / sep_and_peak    cpf.py:241-371  per (K, layer) AUPCs / separability-peakness
* frob                         cpf.py:374-395

Heatmaps come from lrp_ref.subspace_heatmaps (mode "exact" = the kernels' arithmetic), flipping
from flip_ref.flip, both on CPU tensors; the model forward used for flipping is passed in
(``forward_func``), as the product takes the model's own forward.
"""
from __future__ import annotations

import numpy as np
import torch

import flip_ref
import lrp_ref


def heatmaps(model, rules, U, K, layer_idx, x, class_idx, case):
    """HeatmapGenerator(model, U, ..., layer_idx).generate_subspace_heatmaps(x) -> sorted
    subspace heatmaps [b, K, H, W] (numpy float32), exact-order arithmetic."""
    from drsa_audio_amd.model.modify_model import ProjectionModel
    pm = ProjectionModel(model, layer_idx, torch.as_tensor(U, dtype=torch.float32), K, case=case).eval()
    return lrp_ref.subspace_heatmaps(pm, rules, K, x, class_idx=class_idx, mode="exact")["subspace_heatmaps"]


def interclass_concept_flipping(model, x, rules, Us, genres, K, layer_idcs, forward_func, case):
    n = len(genres)
    spc = x.size(0) // n
    out = []
    for layer_idx in layer_idcs:
        aupcs = []
        for i, sub_genre in enumerate(genres):
            U = Us[layer_idx][sub_genre]
            R = []
            for j, _ in enumerate(genres):
                xb = x[i * spc:(i + 1) * spc]          # cpf.py:158 slices with i (D14)
                R.append(heatmaps(model, rules, U, K, layer_idx, xb, j, case))
            R = torch.from_numpy(np.concatenate(R, 0))
            aupc, _, _, _ = flip_ref.flip(forward_func, x, R, 16)
            aupcs.append(aupc.mean(axis=-1))
        out.append(np.stack(aupcs, axis=0))
    return out


def random_projection(dim, permutations=3):
    from scipy.stats import ortho_group
    U = ortho_group.rvs(dim)
    for _ in range(permutations):
        mask = np.random.permutation(dim)
        U = torch.tensor(U[:, mask], dtype=torch.float32)      # cpf.py:214-215
    return U


def cf_random_subspace(model, x, rules, layer_idx, dim, genres, K, case, permutations=3):
    U = random_projection(dim, permutations)
    spc = x.size(0) // len(genres)
    return np.concatenate([heatmaps(model, rules, U, K, layer_idx, x[i * spc:(i + 1) * spc], i, case)
                           for i in range(len(genres))], 0)


def separability_peakness(RU):
    sep_scores = (np.max(RU, 1).sum((-2, -1)) - np.max(RU.sum((-2, -1)), 1)).squeeze()
    peak_scores = np.max(RU, (-2, -1)).sum(1).squeeze()
    sep, peak = sep_scores.mean(), peak_scores.mean()
    return sep, sep / np.sqrt(sep_scores.shape[0]), peak, peak / np.sqrt(peak_scores.shape[0])


def frob(RU, K):
    out = 0.0
    n = 0
    vals = []
    for b in range(RU.shape[0]):
        tot = np.float32(0)
        for k in range(K):
            for l in range(k + 1, K):
                d = (RU[b, l] - RU[b, k]).astype(np.float32)      # RU[:, None] - RU[:, :, None]: [b, k, l] = l - k
                tot = np.float32(tot + np.sqrt(np.sum(d ** 2)))
        vals.append(tot)
    return np.float32(np.mean(np.array(vals, dtype=np.float32))) / (K * (K - 1) / 2)
