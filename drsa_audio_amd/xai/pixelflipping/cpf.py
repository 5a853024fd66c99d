"""Concept flipping and the concept-heatmap metrics, drop-in for ``cxai.xai.pixelflipping.cpf``
(reference cpf.py:20-395):

* ``concept_flipping``             cpf.py:20-84   per class block, the K subspace heatmaps of
                                                  HeatmapGenerator with that class's projection
                                                  matrix; one Flipper pass (patch 16) over the
                                                  balanced batch, the K concepts flipped as a union
* ``interclass_concept_flipping``  cpf.py:87-181  AUPC matrix [subspace genre, attributed genre] per
                                                  layer in [1, 4, 7, 10, 13]
* ``cf_random_subspace``           cpf.py:192-233 subspace heatmaps through a random orthogonal U
                                                  (ortho_group.rvs, column permutations compounding)
* ``perform_cf``                   cpf.py:241-294 AUPC pickles per (K, layer)
* ``sep_and_peak``                 cpf.py:297-371 separability / peakness per (K, layer), pickled
* ``frob``                         cpf.py:374-395 mean pairwise Frobenius distance of concept maps

Heatmaps come from the HIP engine on device.  Where the reference builds one HeatmapGenerator per
(projection matrix, attributed class) over the SAME class batch (interclass, cpf.py:155-163), the
engine runs the forward once and all attributed classes as rows of one backward (per-row class
seeds), since the forward does not depend on the attributed class.

Reference defects handled (new D14-D16):
* D10: ``generate_subspace_heatmaps(concept_flipping=True)`` returns None in the reference (its
  early return is commented out); here the heatmaps come from ``HeatmapGenerator.info_device``
  (concept order does not matter to the Flipper: the K rankings are flipped as a union).
* D14: interclass_concept_flipping slices the class batch with the projection-genre index ``i``
  inside the loop over attributed genres ``j`` (cpf.py:158), so block j of the flipped batch is
  ranked by heatmaps of batch i.  Reproduced by default (``reference_indexing=True``); False
  takes batch j, the documented intent ("samples of a target class").
* D15: perform_cf / sep_and_peak unpack four values from concept_flipping (three are returned)
  and call ``cf_random_subspace`` (which returns heatmaps) as if it returned AUPCs; sep_and_peak
  uses concept_flipping's result as heatmaps.  Intended semantics here: perform_cf's AUPCs come
  from concept flipping with the DRSA (or, prefix 'random', the random) subspaces;
  sep_and_peak's RU are the subspace heatmaps of the same two sources.
* D16: sep_and_peak calls ``frob(RU, num_concepts)`` with the whole list of K values (an error);
  here frob gets the current K (its value is unused by the reference's outputs).
* D17: perform_cf writes to ``os.path.join(out, f'{prefix}/{k}_concepts')``, which for the default
  prefix '' is the absolute path ``/{k}_concepts``; here ``{out}/{prefix}/{k}_concepts``.
* ``case=`` (D5) selects the toy class map as in the reference; HeatmapGenerator infers it from
  the class name.
"""
from __future__ import annotations

import os
import pickle
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from ...engine import get_engine
from ...utils.constants import CLASS_IDX_MAPPER, CLASS_IDX_MAPPER_TOY
from ...utils.evaluation import load_projection_matrix
from ..explain.explainer import HeatmapGenerator
from .core import Flipper

GTZAN_LAYERS = [1, 4, 7, 10, 13]
GTZAN_DIMS = [32, 32, 64, 64, 128]
TOY_DIMS = [8, 8, 16, 16, 16]


def _mapper(case=None, toy=False):
    return CLASS_IDX_MAPPER_TOY if (toy or case == "toy") else CLASS_IDX_MAPPER


def _model_forward(model):
    return lambda b: model(b)                      # the reference's forward_func (cpf.py:79)


def _subspace_heatmaps(model, x, U, name_map, genre, K, layer_idx, device, cls_rows=None) -> torch.Tensor:
    """[b, K, H, W] subspace heatmaps on device (HeatmapGenerator through the engine).  cls_rows:
    optional per-row class indices (the same U, different attributed classes, one pass)."""
    gen = HeatmapGenerator(model, torch.as_tensor(U), name_map, sample_class=genre, num_concepts=K,
                           layer_idx=layer_idx, device=device)
    if cls_rows is None:
        gen.generate_subspace_heatmaps(x, to_host=False)
        return gen.info_device["subspace_heatmaps"]
    eng = get_engine(gen.projectionmodel, gen.composite)
    return eng.subspace_heatmaps(x.to(device, torch.float32).contiguous(), cls=cls_rows)["subspace_heatmaps"]


def concept_flipping(model, input_batch, name_map, layer_idx, path_to_U: Optional[str] = None,
                     num_concepts: int = 4, standard_r: bool = False, case=None,
                     device=torch.device("cuda"), Us: Optional[Dict[str, torch.Tensor]] = None,
                     perturbation_size: int = 16, forward_func=None, return_heatmaps: bool = False):
    """cpf.py:20-84.  ``Us`` (extension) maps class names to matrices instead of a directory of DRSA
    runs; ``return_heatmaps`` also returns the flipped heatmaps [B, K, H, W] (device)."""
    if isinstance(input_batch, np.ndarray):
        input_batch = torch.tensor(input_batch)
    mapper = _mapper(case)
    x = input_batch.to(device)
    spc = x.size(0) // len(mapper)
    heatmaps = []
    for i, genre in enumerate(mapper):
        U = Us[genre] if Us is not None else load_projection_matrix(genre, layer_idx, path_to_U, device=device)
        gen = HeatmapGenerator(model, torch.as_tensor(U), name_map, sample_class=genre, num_concepts=num_concepts,
                               layer_idx=layer_idx, device=device)
        gen.generate_subspace_heatmaps(x[i * spc:(i + 1) * spc], to_host=False)
        key = "standard_heatmaps" if standard_r else "subspace_heatmaps"
        heatmaps.append(gen.info_device[key])
    R = torch.cat(heatmaps, 0)
    flipper = Flipper(perturbation_size=perturbation_size, device=device)
    fwd = forward_func if forward_func is not None else _model_forward(model)
    out = flipper(fwd, x, R)
    return (out + (R,)) if return_heatmaps else out


def interclass_concept_flipping(model, input_batch, name_map, path_to_U: Optional[str] = None, case=None,
                                standard_r: bool = False, toy: bool = False, num_concepts: int = 4,
                                device=torch.device("cuda"), Us: Optional[Dict[int, Dict[str, torch.Tensor]]] = None,
                                layer_idcs: Sequence[int] = tuple(GTZAN_LAYERS), reference_indexing: bool = True,
                                perturbation_size: int = 16, forward_func=None) -> List[np.ndarray]:
    """cpf.py:87-181: for every layer, the [n_classes, n_classes] matrix of class-mean AUPCs whose
    row i uses the projection matrix of genre i and whose column j attributes genre j (D14 on
    which class batch is attributed).  ``Us[layer][genre]`` (extension) replaces the run directory."""
    if isinstance(input_batch, np.ndarray):
        input_batch = torch.tensor(input_batch)
    mapper = {"class1": 0, "class2": 1} if toy else CLASS_IDX_MAPPER
    genres = list(mapper)
    n = len(genres)
    x = input_batch.to(device)
    spc = int(x.size(0) / n)
    flipper = Flipper(perturbation_size=perturbation_size, device=device)
    fwd = forward_func if forward_func is not None else _model_forward(model)
    out = []
    for layer_idx in layer_idcs:
        aupcs = []
        for i, sub_genre in enumerate(genres):
            U = Us[layer_idx][sub_genre] if Us is not None else load_projection_matrix(sub_genre, layer_idx, path_to_U,
                                                                                      device=device)
            if reference_indexing:
                # block j = class batch i attributed to genre j: one forward, n classes as row seeds
                xb = x[i * spc:(i + 1) * spc].repeat(n, 1, 1, 1)
                cls = torch.arange(n, device=device, dtype=torch.int32).repeat_interleave(spc)
                R = _subspace_heatmaps(model, xb, U, name_map, sub_genre, num_concepts, layer_idx, device, cls_rows=cls)
            else:
                R = torch.cat([_subspace_heatmaps(model, x[j * spc:(j + 1) * spc], U, name_map, g, num_concepts,
                                                  layer_idx, device) for j, g in enumerate(genres)], 0)
            aupc, _, _ = flipper(fwd, x, R)
            aupcs.append(aupc.mean(axis=-1))
        out.append(np.stack(aupcs, axis=0))
    return out


def random_projection(dim: int, permutations: int = 3) -> np.ndarray:
    """cf_random_subspace's U (cpf.py:209-215): ortho_group.rvs(dim) from numpy's global RNG, then
    per permutation a column permutation of the previous one (compounding); the last one is the
    one whose heatmaps the reference returns.  Consumes the global RNG exactly as the reference."""
    from scipy.stats import ortho_group
    U = ortho_group.rvs(dim)
    for _ in range(permutations):
        mask = np.random.permutation(dim)
        U = np.asarray(U)[:, mask].astype(np.float32)
    return np.ascontiguousarray(U)


def cf_random_subspace(model, input_batch, name_map, layer_idx, dim, case=None, device=torch.device("cuda"),
                       permutations: int = 3, num_concepts: int = 4, as_tensor: bool = False):
    """cpf.py:192-233: subspace heatmaps [B, K, H, W] (numpy, or the device tensor with
    ``as_tensor``) of every class block through a random orthogonal U.  The reference recomputes
    the heatmaps for each permutation and returns the last; only the last is computed here (the
    RNG is consumed identically)."""
    if isinstance(input_batch, np.ndarray):
        input_batch = torch.tensor(input_batch)
    x = input_batch.to(device)
    mapper = _mapper(case)
    spc = x.size(0) // len(mapper)
    U = torch.tensor(random_projection(dim, permutations), dtype=x.dtype, device=device) if permutations > 0 else \
        torch.tensor(__import__("scipy.stats", fromlist=["ortho_group"]).ortho_group.rvs(dim), dtype=x.dtype,
                     device=device)
    R = torch.cat([_subspace_heatmaps(model, x[i * spc:(i + 1) * spc], U, name_map, g, num_concepts, layer_idx, device)
                   for i, g in enumerate(mapper)], 0)
    return R if as_tensor else R.cpu().numpy()


def _subspace_source(model, x, name_map, layer_idx, k, dim, prefix, path, case, device):
    """RU for one (K, layer): DRSA subspaces from ``path/{k}_concepts`` runs, or random ones."""
    if prefix == "random":
        return cf_random_subspace(model, x, name_map, layer_idx, dim=dim, case=case, device=device, permutations=3,
                                  num_concepts=k, as_tensor=True)
    _, _, _, R = concept_flipping(model, x, name_map, layer_idx, os.path.join(path, f"{k}_concepts"), num_concepts=k,
                                  case=case, device=device, return_heatmaps=True)
    return R


def perform_cf(model, input_batch, name_map, out, path=None, layer_idcs=(1, 4, 7, 10, 13), num_concepts=(2, 4, 8, 16),
               toy=False, prefix="", device=torch.device("cuda")):
    """cpf.py:241-294: AUPC per instance [n_classes, samples_per_class] for every (K, layer),
    pickled to ``{out}/{prefix}/{K}_concepts/aupcs_layer_{L}.pkl`` (D15)."""
    dims = TOY_DIMS if toy else GTZAN_DIMS
    case = "toy" if toy else None
    x = (torch.tensor(input_batch) if isinstance(input_batch, np.ndarray) else input_batch).to(device)
    res = {}
    for k in num_concepts:
        for i, layer_idx in enumerate(layer_idcs):
            print(f"Performing concept patch flipping for {k} subspaces at layer {layer_idx}")
            if prefix == "random":
                R = _subspace_source(model, x, name_map, layer_idx, k, dims[i], prefix, path, case, device)
                aupc, _, _ = Flipper(perturbation_size=16, device=device)(_model_forward(model), x, R)
            else:
                aupc, _, _ = concept_flipping(model, x, name_map, layer_idx, os.path.join(path, f"{k}_concepts"),
                                              num_concepts=k, case=case, device=device)
            conf_out = os.path.join(out, prefix, f"{k}_concepts")   # D17
            os.makedirs(conf_out, exist_ok=True)
            with open(os.path.join(conf_out, f"aupcs_layer_{layer_idx}.pkl"), "wb") as fh:
                pickle.dump(np.stack(aupc, axis=0), fh)
            res[(k, layer_idx)] = aupc
    return res


def separability_peakness(RU: np.ndarray):
    """sep_and_peak's per-(K, layer) numbers from heatmaps RU [b, K, H, W] (cpf.py:348-354):
    separability = mean_b( sum_hw max_k RU - max_k sum_hw RU ), peakness = mean_b( sum_k max_hw RU ),
    each with the reference's 'standard error' (value / sqrt(b))."""
    sep_scores = (np.max(RU, 1).sum((-2, -1)) - np.max(RU.sum((-2, -1)), 1)).squeeze()
    sep = sep_scores.mean()
    peak_scores = np.max(RU, (-2, -1)).sum(1).squeeze()
    peak = peak_scores.mean()
    return sep, sep / np.sqrt(sep_scores.shape[0]), peak, peak / np.sqrt(peak_scores.shape[0])


def sep_and_peak(model, input_batch, name_map, out, path=None, layer_idcs=(1, 4, 7, 10, 13),
                 num_concepts=(2, 4, 8, 16), toy=False, prefix="", device=torch.device("cuda")) -> np.ndarray:
    """cpf.py:297-371: [len(num_concepts), 4 (sep, sep_err, peak, peak_err), len(layer_idcs)],
    pickled to ``{out}/{prefix}/sep_and_peak.pkl`` (D15, D16)."""
    dims = TOY_DIMS if toy else GTZAN_DIMS
    case = "toy" if toy else None
    x = (torch.tensor(input_batch) if isinstance(input_batch, np.ndarray) else input_batch).to(device)
    allk = []
    for k in num_concepts:
        sep, seperr, peak, peakerr = [], [], [], []
        for i, layer_idx in enumerate(layer_idcs):
            print(f"Performing concept patch flipping for {k} subspaces at layer {layer_idx}")
            RU = _subspace_source(model, x, name_map, layer_idx, k, dims[i], prefix,
                                  None if path is None else os.path.join(path, prefix), case, device).cpu().numpy()
            frob(RU, k)                                    # computed as the reference does; unused (D16)
            s, se, p, pe = separability_peakness(RU)
            sep.append(s)
            seperr.append(se)
            peak.append(p)
            peakerr.append(pe)
        allk.append(np.stack((sep, seperr, peak, peakerr), axis=0))
    final = np.stack(allk, axis=0)
    conf_out = os.path.join(out, f"{prefix}")
    os.makedirs(conf_out, exist_ok=True)
    with open(os.path.join(conf_out, "sep_and_peak.pkl"), "wb") as fh:
        pickle.dump(np.stack(final, axis=0), fh)
    return final


def frob(RU: np.ndarray, num_concepts: int) -> float:
    """cpf.py:374-395: mean over samples of sum_{k<l} ||RU_k - RU_l||_F, divided by K(K-1)/2."""
    diff = RU[:, None, :, :, :] - RU[:, :, None, :, :]
    fro_norms = np.sqrt(np.sum(diff ** 2, axis=(-2, -1)))
    mask = np.triu(np.ones((num_concepts, num_concepts), dtype=bool), k=1)
    total = np.sum(fro_norms[:, mask], axis=-1)
    return total.mean() / (num_concepts * (num_concepts - 1) / 2)
