"""LRP attribution entry points, drop-in for ``cxai.xai.explain.attribute``.

* ``SubspaceHook``         — reference attribute.py:12-67 (relevance mask per subspace clone)
* ``compute_relevances``   — reference attribute.py:70-108
* ``lrp_output_modifier``  — reference attribute.py:111-160

``compute_relevances`` runs the compiled HIP plan (forward with fused rule denominators,
rule backward per layer) through the zennit-compatible ``Gradient`` attributor.
"""
from __future__ import annotations

from typing import Tuple

import torch
import torch.nn as nn

from ...zennit.attribution import Gradient
from ...zennit.composites import Composite
from ...zennit.core import Hook


class SubspaceHook(Hook):
    """Masks the relevance of clone k (k = 1..K) of every K+1 consecutive rows to subspace
    k-1; clone 0 keeps all subspaces.  The HIP engine executes this mask inside the fused
    projection backward (``drsa_amd_projection_bwd``); ``backward`` below is the same
    arithmetic on a tensor, kept for API parity."""

    def __init__(self, num_concepts: int = 4, stabilizer: float = 1e-7,
                 device: str | torch.device = torch.device("cpu")) -> None:
        super().__init__()
        self.num_concepts = int(num_concepts)
        self.stabilizer = stabilizer
        self.device = torch.device(device) if isinstance(device, str) else device

    def backward(self, module, grad_input, grad_output) -> Tuple[torch.Tensor]:
        g, = grad_output
        b, n, c, dk = g.size()
        K = self.num_concepts
        eye = torch.eye(K, device=g.device, dtype=g.dtype)
        gv = g.reshape(-1, K + 1, n, c, dk)
        masked = torch.cat([gv[:, :1], gv[:, 1:] * eye[None, :, None, :, None]], dim=1)
        return (masked.reshape(b, n, c, dk),)

    def copy(self):
        return self.__class__(num_concepts=self.num_concepts, stabilizer=self.stabilizer, device=self.device)


def compute_relevances(model: nn.Module, input_batch: torch.Tensor, composite: Composite,
                       num_classes: int = None, class_idx: int = None,
                       one_hot_encoded: bool = False) -> torch.Tensor:
    """LRP heatmaps of ``input_batch`` (same shape as the input)."""
    with Gradient(model, composite) as attributor:
        _, relevance = attributor(input_batch, lrp_output_modifier(class_idx, num_classes, one_hot_encoded))
    return relevance


def lrp_output_modifier(class_idx: int = None, num_classes: int = None, one_hot_encoded: bool = False):
    """Output-relevance seed: logits (or 1) at ``class_idx``, or the block-diagonal
    all-classes mask for a class-balanced, class-ordered batch."""
    assert class_idx is not None or num_classes is not None, \
        "Provide either class_idx to attribute or samples_per_class to be able to build attribution mask for batch"
    if class_idx is not None:
        def extract_output_class(output):
            mask = torch.zeros_like(output)
            mask[..., class_idx] = 1
            return mask if one_hot_encoded else output * mask
        return extract_output_class

    def attribute_all_classes(output):
        per = output.size(0) // num_classes
        if per * num_classes != output.size(0):
            # reference defect D8: repeat_interleave would produce a size mismatch
            raise ValueError(f"batch of {output.size(0)} is not divisible by num_classes={num_classes}")
        mask = torch.repeat_interleave(torch.eye(num_classes, device=output.device, dtype=output.dtype), per, dim=0)
        return mask if one_hot_encoded else output * mask
    return attribute_all_classes


def seed_class_indices(batch: int, class_idx: int = None, num_classes: int = None, device=None) -> torch.Tensor:
    """The row -> attributed class map of ``lrp_output_modifier`` as int32 indices, the form the
    fused seed of ``drsa_amd_linear_bwd`` takes: ``class_idx`` for every row, or (all-classes mode)
    row b -> b // (batch / num_classes), the rows of ``repeat_interleave(eye(C), batch // C)``
    (attribute.py:152).  A batch not divisible by num_classes raises, as the reference's mask
    does (D8)."""
    if class_idx is not None:
        return torch.full((batch,), int(class_idx), device=device, dtype=torch.int32)
    if num_classes is None:
        raise ValueError("Provide either class_idx to attribute or num_classes")
    per = batch // num_classes
    if per * num_classes != batch:
        raise ValueError(f"batch of {batch} is not divisible by num_classes={num_classes}")
    return torch.arange(num_classes, device=device, dtype=torch.int32).repeat_interleave(per)
