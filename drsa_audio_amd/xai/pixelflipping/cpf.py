"""Concept flipping, drop-in for ``cxai.xai.pixelflipping.cpf.concept_flipping`` (reference
cpf.py:20-80): per class block, the K subspace heatmaps of HeatmapGenerator with that class's
projection matrix, then one Flipper pass (patch size 16) over the whole balanced batch with the
K concepts of each sample flipped as a union.

Differences from the reference (defect D5 in SURVEY.md: the reference passes a non-existent
``case=`` kwarg and relies on a commented-out ``concept_flipping`` branch of
generate_subspace_heatmaps): the heatmaps are taken from ``HeatmapGenerator.info_device``;
``Us`` may map class names to matrices instead of a directory of DRSA runs.
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np
import torch

from ...utils.constants import CLASS_IDX_MAPPER, CLASS_IDX_MAPPER_TOY
from ...utils.evaluation import load_projection_matrix
from ..explain.explainer import HeatmapGenerator
from .core import Flipper


def concept_flipping(model, input_batch, name_map, layer_idx, path_to_U: Optional[str] = None,
                     num_concepts: int = 4, standard_r: bool = False, case=None,
                     device=torch.device("cuda"), Us: Optional[Dict[str, torch.Tensor]] = None,
                     perturbation_size: int = 16, forward_func=None):
    if isinstance(input_batch, np.ndarray):
        input_batch = torch.tensor(input_batch)
    mapper = CLASS_IDX_MAPPER if case != "toy" else CLASS_IDX_MAPPER_TOY
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
    fwd = forward_func if forward_func is not None else (lambda b: model(b))
    return flipper(fwd, x, R)
