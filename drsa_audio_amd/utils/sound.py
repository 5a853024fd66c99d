"""Waveform helpers of the reference (``cxai/utils/sound.py``) on device tensors.

``get_slice`` is pure indexing (a strided view, as the reference's ``unfold``) and
``peak_normalizer`` one elementwise op; the fused HIP front end
(``dataloading.Loader.load_songs``) performs both inside its single launch, so these two exist
for callers that use them on their own.
"""
from __future__ import annotations

import math

import torch


def round_down(n: float, decimalpoints: int) -> float:
    """cxai/utils/utilities.py:6-16."""
    return math.floor(n * 10 ** decimalpoints) / 10 ** decimalpoints


def chunk_hop(slice_length: float, num_chunks: int, sample_rate: int) -> int:
    """Step between get_slice chunks (sound.py:33): evenly spaced over the first 29 s."""
    return int(round_down(((29 - slice_length) / (num_chunks - 1)), 1) * sample_rate)


def get_slice(wav: torch.Tensor, slice_length: float = 6, start_point: float = 0, num_chunks: int = 1,
              sample_rate: int = 16000) -> torch.Tensor:
    """sound.py:8-44.  wav [channels, T] -> [channels*num_chunks, 1, window] (num_chunks > 1) or
    [channels, window]."""
    wav = torch.as_tensor(wav)
    window = int(slice_length * sample_rate)
    if num_chunks > 1:
        hop = chunk_hop(slice_length, num_chunks, sample_rate)
        out = wav[:, :29 * sample_rate].unfold(1, window, hop).reshape(-1, 1, window)
        assert out.shape[0] == num_chunks, "not equal num_chunks"
        return out
    start = int(start_point * sample_rate)
    assert start_point <= wav.size(1) - window, f"Start_point has to be in range [0,{wav.size(1) - window}]"
    return wav[:, start:start + window]


def peak_normalizer(wav: torch.Tensor) -> torch.Tensor:
    """sound.py:67-70: amplitudes scaled into [-1, 1] by the peak along the last axis."""
    wav = torch.as_tensor(wav)
    return wav / torch.abs(wav).max(dim=-1, keepdim=True)[0]
