"""Seeded synthetic inputs for benchmarks, smoke runs and tests (no reference code involved).

``drsa_inputs`` builds DRSA activation / context rows the way the reference's data scripts
shape them: A post-ReLU-like (|N(0,1)|), C signed, both normalised with
``preprocessing.normalize_vectors`` semantics (v / rms / d^{1/4};
/root/reference/cxai/xai/drsa/preprocessing.py normalize_vectors, getdrsadata.py:47-59).
numpy ``default_rng`` (PCG64) is stable across numpy versions, so fixtures made from these rows
in the build container can be regenerated from the seed anywhere.
"""
from __future__ import annotations

import numpy as np
import torch


def drsa_inputs(N: int, d: int, seed: int):
    """(A, C) float32 [N, d]: A = |N(0,1)|, C ~ N(0,1), each divided by its global rms and d^{1/4}."""
    rng = np.random.default_rng(seed)
    A = np.abs(rng.standard_normal((N, d))).astype(np.float32)
    C = rng.standard_normal((N, d)).astype(np.float32)

    def norm(v):
        t = torch.from_numpy(v)
        E = torch.sqrt(torch.mean(torch.square(t)))
        return (t / E / d ** 0.25).numpy()
    return norm(A), norm(C)


def synthetic_songs(n_songs: int, seconds: float = 29.5, sample_rate: int = 16000, seed: int = 0) -> np.ndarray:
    """Music-like synthetic waveforms: a few harmonic tones with vibrato and decaying
    envelopes plus coloured noise, random gain per song.  float32 [S, T]."""
    rng = np.random.default_rng(seed)
    T = int(seconds * sample_rate)
    t = np.arange(T) / sample_rate
    out = np.empty((n_songs, T), dtype=np.float32)
    for i in range(n_songs):
        x = np.zeros(T)
        for _ in range(4):
            f0 = rng.uniform(60, 1500)
            vib = 1 + 0.003 * np.sin(2 * np.pi * rng.uniform(3, 7) * t)
            env = np.exp(-((t * rng.uniform(0.5, 4)) % 1.0) * rng.uniform(1, 6))
            for h in range(1, 6):
                if f0 * h < 7800:
                    x += rng.uniform(0.1, 1) / h * env * np.sin(2 * np.pi * f0 * h * t * vib + rng.uniform(0, 6.3))
        noise = np.cumsum(rng.standard_normal(T)) * 1e-3
        noise -= np.convolve(noise, np.ones(64) / 64, mode="same")
        x += noise + 0.02 * rng.standard_normal(T)
        out[i] = (x * rng.uniform(0.05, 0.9) / np.abs(x).max()).astype(np.float32)
    return out
