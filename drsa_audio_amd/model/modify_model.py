"""Virtual DRSA layers inserted after feature layer ``j`` of a VGG-type CNN.

API mirrors ``cxai.model.modify_model``:

* ``ProjectionModel``  — reference ``cxai/model/modify_model.py:4-60``
* ``SubspaceFilter``   — reference ``cxai/model/modify_model.py:63-72``
* ``Projection``       — reference ``cxai/model/modify_model.py:75-96``  (h = a·U, viewed [b, n, K, d_k])
* ``InvProjection``    — reference ``cxai/model/modify_model.py:99-123`` (a' = h·Uᵀ, back to [b, d, H, W])

These modules carry the layer names the name maps refer to
(``features.projection``, ``features.subspacefilter``, ``features.invprojection``).
The HIP engine (``drsa_audio_amd.engine``) recognises them structurally and runs
the projection forward and the ε/mask/ε relevance backward as fused kernels; the
PyTorch ``forward`` methods below are only the model definition.
"""
from __future__ import annotations

import torch
import torch.nn as nn

__all__ = ["ProjectionModel", "SubspaceFilter", "Projection", "InvProjection"]


class SubspaceFilter(nn.Module):
    """Identity; the subspace relevance mask is attached to it by the composite."""

    def forward(self, act_map: torch.Tensor) -> torch.Tensor:
        return act_map


class Projection(nn.Module):
    """a [b, d, H, W] -> h [b, H*W, K, d_k] with h = a_vec · U."""

    def __init__(self, U: torch.Tensor, num_concepts: int) -> None:
        super().__init__()
        self.U = U
        self.num_concepts = int(num_concepts)
        self.d_k = U.size(0) // self.num_concepts

    def forward(self, act_map: torch.Tensor) -> torch.Tensor:
        b, d = act_map.size(0), act_map.size(1)
        vecs = act_map.reshape(b, d, -1).transpose(1, 2)
        h = vecs @ self.U.to(act_map)
        return h.reshape(b, vecs.size(1), self.num_concepts, self.d_k)


class InvProjection(nn.Module):
    """h [b, n, K, d_k] -> a' [b, d, sqrt(n), sqrt(n)] with a' = h · Uᵀ (square maps, as the reference)."""

    def __init__(self, U: torch.Tensor, num_concepts: int) -> None:
        super().__init__()
        self.U_inv = U.T
        self.num_concepts = int(num_concepts)
        self.d = self.U_inv.size(0)
        self.d_k = self.d // self.num_concepts

    def forward(self, h: torch.Tensor) -> torch.Tensor:
        b, n = h.size(0), h.size(1)
        side = int(round(n ** 0.5))
        a = h.reshape(b, n, self.d) @ self.U_inv.to(h)
        return a.transpose(1, 2).reshape(b, self.d, side, side).contiguous()


class ProjectionModel(nn.Module):
    """Copy of ``model`` with Projection -> SubspaceFilter -> InvProjection inserted
    right after ``model.features[layer_idx]``.

    ``case`` selects the flattened width between trunk and head exactly like the
    reference (2048 for 'gtzan', 64 for 'toy'); ``num_flat_features`` may be given
    explicitly for other models.
    """

    def __init__(self, model: nn.Module, layer_idx: int, U: torch.Tensor,
                 num_concepts: int, case: str = "gtzan",
                 num_flat_features: int | None = None) -> None:
        super().__init__()
        n_feat = len(model.features)
        if not (0 < layer_idx < n_feat):
            raise ValueError(f"layer_idx must be in (0, {n_feat})")
        if num_flat_features is None:
            num_flat_features = 2048 if case == "gtzan" else 64
        self.num_flat_features = int(num_flat_features)
        self.layer_idx = int(layer_idx)
        self.num_concepts = int(num_concepts)
        self.U = U
        self.features = nn.Sequential()
        for idx, layer in enumerate(model.features.children()):
            if idx == layer_idx + 1:
                self.features.add_module("projection", Projection(U, num_concepts))
                self.features.add_module("subspacefilter", SubspaceFilter())
                self.features.add_module("invprojection", InvProjection(U, num_concepts))
            self.features.add_module(str(idx), layer)
        self.classifier = nn.Sequential()
        for idx, layer in enumerate(model.classifier.children()):
            self.classifier.add_module(str(idx), layer)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = self.features(x)
        return self.classifier(x.reshape(-1, self.num_flat_features))
