"""CPU oracle for the log-mel front end.  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
and only as the checker; the product path (drsa_audio_amd.utils.dataloading) never does.

Restates, in numpy float64 (mode "f64") and in torch float32 (mode "torch32"):

* cxai/utils/sound.py:8-44      get_slice (evenly spaced chunks via unfold, or one slice)
* cxai/utils/sound.py:67-70     peak_normalizer (wav / max|wav| along the last axis)
* cxai/utils/utilities.py:6-16  round_down
* cxai/utils/dataloading.py:28-74   Loader.__init__: torchaudio Spectrogram(n_fft, hop, power=None)
                                    + MelScale(n_mels, n_stft=n_fft//2+1, sample_rate)
* cxai/utils/dataloading.py:138-176 Loader.transform_wav: |STFT| -> mel -> log10(+1e-7)
                                    -> clamp(-4) -> frames 1..width

The STFT and mel filterbank are third-party code (torchaudio 2.5.1, requirements.txt:18),
absent from this image.  Their published algorithm is restated here:

* Spectrogram: torch.stft(center=True, pad_mode="reflect", window=hann_window(n_fft,
  periodic=True), onesided, normalized=False, return_complex=True).
* melscale_fbanks(n_freqs, f_min=0, f_max=sr//2, n_mels, sr, norm=None, mel_scale="htk"):
  all_freqs = linspace(0, sr//2, n_freqs); m_pts = linspace(hz2mel(f_min), hz2mel(f_max),
  n_mels+2); f_pts = mel2hz(m_pts); hz2mel(f) = 2595*log10(1+f/700);
  fb = max(0, min(-slopes[:, :-2]/f_diff[:-1], slopes[:, 2:]/f_diff[1:])),
  slopes = f_pts[None] - all_freqs[:, None]; MelScale: mel = (spec^T @ fb)^T.

PARITY STATUS: unpinned vs torchaudio (no torchaudio here and no reference fixture holds a
spectrogram).  The restatement is pinned by known-answer tests instead: the float64 and
float32 (torch.stft) restatements agree, a pure tone lands in the filter whose centre is
nearest, the filterbank's triangles peak at f_pts, and the slicing matches get_slice's
unfold arithmetic (tests/test_oracle_logmel.py).
"""
from __future__ import annotations

import math

import numpy as np
import torch

# cxai/utils/constants.py:7-24 (AUDIO_PARAMS)
AUDIO_PARAMS = {
    "gtzan": {"sample_rate": 16000, "slice_length": 3, "num_chunks": 8, "n_fft": 800, "hop_length": 360,
              "n_mels": 128, "mel_width": 128},
    "toy": {"sample_rate": 16000, "slice_length": 1, "num_chunks": 1, "n_fft": 480, "hop_length": 240,
            "n_mels": 64, "mel_width": 64},
}


def round_down(n: float, decimalpoints: int) -> float:
    """utilities.py:6-16."""
    return math.floor(n * 10 ** decimalpoints) / 10 ** decimalpoints


def get_slice(wav: np.ndarray, slice_length=6, start_point=0, num_chunks=1, sample_rate=16000) -> np.ndarray:
    """sound.py:8-44.  wav [channels, T] -> [num_chunks*channels, 1, window] (num_chunks > 1)
    or [channels, window] (single slice)."""
    window = int(slice_length * sample_rate)
    if num_chunks > 1:
        hop = int(round_down((29 - slice_length) / (num_chunks - 1), 1) * sample_rate)
        w = wav[:, :29 * sample_rate]
        n = (w.shape[1] - window) // hop + 1
        out = np.stack([w[:, i * hop:i * hop + window] for i in range(n)], axis=1)   # [ch, n, window]
        out = out.reshape(-1, 1, window)
        assert out.shape[0] == num_chunks * wav.shape[0] or wav.shape[0] != 1 or n == num_chunks
        return out
    start = int(start_point * sample_rate)
    assert start_point <= wav.shape[1] - window
    return wav[:, start:start + window]


def chunk_hop(slice_length: float, num_chunks: int, sample_rate: int) -> int:
    """The unfold step of get_slice (sound.py:33)."""
    return int(round_down((29 - slice_length) / (num_chunks - 1), 1) * sample_rate)


def peak_normalizer(wav):
    """sound.py:67-70."""
    return wav / np.abs(wav).max(axis=-1, keepdims=True)


def hz_to_mel(f):
    return 2595.0 * math.log10(1.0 + f / 700.0)


def melscale_fbanks(n_freqs, f_min, f_max, n_mels, sample_rate, mode="f64"):
    """torchaudio.functional.melscale_fbanks (htk, norm=None) -> [n_freqs, n_mels]."""
    if mode == "torch32":
        all_freqs = torch.linspace(0, sample_rate // 2, n_freqs)
        m_pts = torch.linspace(hz_to_mel(f_min), hz_to_mel(f_max), n_mels + 2)
        f_pts = 700.0 * (10.0 ** (m_pts / 2595.0) - 1.0)
        f_diff = f_pts[1:] - f_pts[:-1]
        slopes = f_pts.unsqueeze(0) - all_freqs.unsqueeze(1)
        down = (-1.0 * slopes[:, :-2]) / f_diff[:-1]
        up = slopes[:, 2:] / f_diff[1:]
        return torch.max(torch.zeros(1), torch.min(down, up)).numpy()
    all_freqs = np.linspace(0, sample_rate // 2, n_freqs)
    m_pts = np.linspace(hz_to_mel(f_min), hz_to_mel(f_max), n_mels + 2)
    f_pts = 700.0 * (10.0 ** (m_pts / 2595.0) - 1.0)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts[None, :] - all_freqs[:, None]
    down = -slopes[:, :-2] / f_diff[:-1]
    up = slopes[:, 2:] / f_diff[1:]
    return np.maximum(0.0, np.minimum(down, up))


def filter_centres(f_min, f_max, n_mels):
    m_pts = np.linspace(hz_to_mel(f_min), hz_to_mel(f_max), n_mels + 2)
    return 700.0 * (10.0 ** (m_pts / 2595.0) - 1.0)


def stft_mag(wav: np.ndarray, n_fft: int, hop: int, mode="f64") -> np.ndarray:
    """|Spectrogram(n_fft, hop, power=None)(wav)| -> [..., n_fft//2+1, 1 + T//hop]."""
    if mode == "torch32":
        x = torch.from_numpy(np.ascontiguousarray(wav, dtype=np.float32))
        shp = x.shape
        x = x.reshape(-1, shp[-1])
        X = torch.stft(x, n_fft, hop_length=hop, win_length=n_fft, window=torch.hann_window(n_fft),
                       center=True, pad_mode="reflect", normalized=False, onesided=True, return_complex=True)
        return X.abs().reshape(*shp[:-1], X.shape[-2], X.shape[-1]).numpy()
    x = np.asarray(wav, dtype=np.float64)
    shp = x.shape
    x = x.reshape(-1, shp[-1])
    pad = n_fft // 2
    xp = np.pad(x, ((0, 0), (pad, pad)), mode="reflect")
    T = 1 + shp[-1] // hop
    win = 0.5 - 0.5 * np.cos(2.0 * np.pi * np.arange(n_fft) / n_fft)
    idx = np.arange(T)[:, None] * hop + np.arange(n_fft)[None, :]
    frames = xp[:, idx] * win                                     # [b, T, n_fft]
    X = np.fft.rfft(frames, axis=-1)                              # [b, T, n_freq]
    return np.abs(X).transpose(0, 2, 1).reshape(*shp[:-1], n_fft // 2 + 1, T)


def mel_spectrogram(wav, n_fft, hop, n_mels, sample_rate, mode="f64"):
    mag = stft_mag(wav, n_fft, hop, mode)                         # [..., F, T]
    fb = melscale_fbanks(n_fft // 2 + 1, 0.0, float(sample_rate // 2), n_mels, sample_rate, mode)
    if mode == "torch32":
        m = torch.from_numpy(mag)
        return torch.matmul(m.transpose(-1, -2), torch.from_numpy(fb)).transpose(-1, -2).numpy()
    return np.swapaxes(np.swapaxes(mag, -1, -2) @ fb, -1, -2)


def transform_wav(wav, case="gtzan", clamp=True, mode="f64"):
    """Loader(case).transform_wav(wav) -> [-1, 1, n_mels, width] (dataloading.py:138-176)."""
    p = AUDIO_PARAMS[case]
    mel = mel_spectrogram(wav, p["n_fft"], p["hop_length"], p["n_mels"], p["sample_rate"], mode)
    logmel = np.log10(mel + (1e-7 if mode == "f64" else np.float32(1e-7)))
    if clamp:
        logmel = np.maximum(logmel, -4)
    logmel = logmel[..., 1:p["mel_width"] + 1]
    assert logmel.shape[-1] == p["mel_width"]
    return logmel.reshape(-1, 1, p["n_mels"], p["mel_width"])


def load_songs(songs: np.ndarray, case="gtzan", num_chunks=None, mode="f64"):
    """Loader.load for in-memory songs [S, T]: get_slice -> peak_normalizer -> transform_wav
    (dataloading.py:76-111), one [num_chunks, 1, n_mels, width] block per song."""
    p = AUDIO_PARAMS[case]
    nc = p["num_chunks"] if num_chunks is None else num_chunks
    out = []
    for s in songs:
        w = get_slice(s[None, :], p["slice_length"], 0, nc, p["sample_rate"])
        w = peak_normalizer(np.asarray(w, dtype=np.float64 if mode == "f64" else np.float32))
        out.append(transform_wav(w, case, True, mode))
    return np.concatenate(out, axis=0)


# the synthetic songs generator moved to the product's data module (bench.py may not import the oracle)
from drsa_audio_amd.utils.synthetic import synthetic_songs  # noqa: E402,F401
