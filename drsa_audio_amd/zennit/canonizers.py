"""Canonizers (zennit.canonizers).  ``SequentialMergeBatchNorm`` folds every BatchNorm that
directly follows a Conv2d/Linear into it (w' = w·γ/√(σ²+ε), b' = (b−μ)·γ/√(σ²+ε) + β),
as zennit's MergeBatchNorm does; the engine applies it to its private weight copies at plan
compile time (the user's model is not modified)."""
from __future__ import annotations

import torch


class Canonizer:
    def apply(self, root_module):
        return []

    def copy(self):
        return self.__class__()


class SequentialMergeBatchNorm(Canonizer):
    kind = "merge_bn"

    @staticmethod
    @torch.no_grad()
    def fold(weight: torch.Tensor, bias, bn) -> tuple:
        denominator = (bn.running_var + bn.eps) ** 0.5
        scale = bn.weight / denominator
        shape = (-1,) + (1,) * (weight.dim() - 1)
        w = weight * scale.reshape(shape)
        b0 = bias if bias is not None else torch.zeros_like(bn.running_mean)
        b = (b0 - bn.running_mean) * scale + bn.bias
        return w, b


MergeBatchNorm = SequentialMergeBatchNorm
