"""VGG-type audio CNN factory (the model family the LRP/DRSA path explains).

Mirrors the constructor API of ``cxai.model.create_model`` so that checkpoints
and name maps written for the reference load unchanged:

* ``VGGType``                  — reference ``cxai/model/create_model.py:8-97``
* ``get_conv_block_layers``    — reference ``cxai/model/create_model.py:100-137``
* ``get_dense_block_layers``   — reference ``cxai/model/create_model.py:140-171``
* ``get_out_shape``            — reference ``cxai/model/create_model.py:174-211``

Module creation order (and therefore PyTorch default initialisation under a
fixed ``torch.manual_seed``) is identical to the reference; this is pinned by
``tests/golden/model_fixture.npz`` (see ``oracle/gen_fixtures.py``).

The ``forward`` here is a plain PyTorch forward kept for users who want logits;
the explanation hot path never calls it — it is compiled into a HIP plan by
``drsa_audio_amd.engine``.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import torch
import torch.nn as nn

__all__ = ["VGGType", "get_conv_block_layers", "get_dense_block_layers",
           "get_out_shape", "num_flat_features"]


def _pair(k) -> Tuple[int, int]:
    return (int(k), int(k)) if isinstance(k, int) else (int(k[0]), int(k[1]))


def get_conv_block_layers(n_in: int, n_out: int, block_depth: int = 2,
                          kernel=(3, 3), stride: int = 1, padding=1,
                          padding_mode: str = "zeros",
                          conv_bn: bool = True) -> List[nn.Module]:
    """``block_depth`` x (Conv2d -> [BatchNorm2d] -> ReLU)."""
    out: List[nn.Module] = []
    channels = n_in
    for _ in range(block_depth):
        out.append(nn.Conv2d(channels, n_out, kernel_size=kernel, stride=stride,
                             padding=padding, padding_mode=padding_mode))
        if conv_bn:
            out.append(nn.BatchNorm2d(num_features=n_out))
        out.append(nn.ReLU())
        channels = n_out
    return out


def get_dense_block_layers(n_in: int, n_out: int, dropout: float,
                           depth: int = 2, dense_bn: bool = True) -> List[nn.Module]:
    """``depth`` x (Linear -> [BatchNorm1d] -> ReLU -> [Dropout])."""
    out: List[nn.Module] = []
    width = n_in
    for _ in range(depth):
        out.append(nn.Linear(in_features=width, out_features=n_out))
        if dense_bn:
            out.append(nn.BatchNorm1d(n_out))
        out.append(nn.ReLU())
        if dropout:
            out.append(nn.Dropout(dropout))
        width = n_out
    return out


def get_out_shape(input_size=(128, 216), conv_kernel=(3, 3),
                  pool_kernels=((4, 4), (2, 4), (2, 2), (2, 2)),
                  out_filters: int = 128, padding=1, stride: int = 1,
                  block_depth: int = 2) -> int:
    """Flattened feature size after the conv trunk (same arithmetic as the reference)."""
    pad = 1 if padding == "same" else (0 if isinstance(padding, str) else int(padding))
    h, w = float(input_size[0]), float(input_size[1])
    for pk in pool_kernels:
        ph, pw = _pair(pk)
        for _ in range(block_depth):
            h = (h - conv_kernel[0] + 2 * pad) / stride + 1
            w = (w - conv_kernel[1] + 2 * pad) / stride + 1
        h = int((h - (ph - 1) - 1) / ph + 1)
        w = int((w - (pw - 1) - 1) / pw + 1)
    return int(h * w * out_filters)


def num_flat_features(x: torch.Tensor) -> int:
    n = 1
    for s in x.size()[1:]:
        n *= s
    return n


class VGGType(nn.Module):
    """Configurable VGG-style CNN: ``features`` (conv blocks + max-pool) and ``classifier``.

    Same argument names and defaults as the reference constructor.
    """

    def __init__(self, n_filters: Sequence[int] = (32, 64, 96, 128),
                 conv_kernel=(3, 3),
                 pool_kernels=((4, 4), (2, 4), (2, 2), (2, 2)),
                 n_dense: int = 512, n_classes: int = 10, dropout: float = 0.2,
                 block_depth: int = 2, dense_depth: int = 2,
                 input_size=(128, 256), padding="same", stride: int = 1,
                 conv_bn: bool = True, dense_bn: bool = True) -> None:
        super().__init__()
        if len(n_filters) != len(pool_kernels):
            raise ValueError("number of conv blocks and max-pool kernels must match")
        trunk: List[nn.Module] = []
        prev = 1
        for width, pk in zip(n_filters, pool_kernels):
            trunk += get_conv_block_layers(prev, width, block_depth=block_depth,
                                           kernel=conv_kernel, stride=stride,
                                           padding=padding, conv_bn=conv_bn)
            trunk.append(nn.MaxPool2d(pk))
            prev = width
        self.features = nn.Sequential(*trunk)
        flat = get_out_shape(input_size=input_size, conv_kernel=conv_kernel,
                             pool_kernels=pool_kernels, padding=padding,
                             out_filters=n_filters[-1], block_depth=block_depth)
        self.num_flat_features = flat
        head = get_dense_block_layers(flat, n_dense, dropout=dropout,
                                      depth=dense_depth, dense_bn=dense_bn)
        head.append(nn.Linear(n_dense, n_classes))
        self.classifier = nn.Sequential(*head)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        # The reference hard-codes view(-1, 2048) (create_model.py:95, defect D6);
        # the flattened size is derived from the configuration here.
        x = self.features(x)
        return self.classifier(x.reshape(x.size(0), -1))
