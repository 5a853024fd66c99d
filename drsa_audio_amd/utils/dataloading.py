"""Log-mel front end: the reference's ``Loader`` (``cxai/utils/dataloading.py:13-176``) on the
HIP kernel ``drsa_amd_logmel`` (``csrc/logmel.hip``).

``Loader(case)`` builds the transform tables once on the device: the analysis window
(``torch.hann_window(n_fft)``, periodic, as torchaudio ``Spectrogram``) and the HTK mel
filterbank (torchaudio ``melscale_fbanks``, norm=None, restated below in the same float32
torch arithmetic) in band form.  ``transform_wav`` is the reference's method of the same
name; ``load_songs`` fuses ``get_slice`` + ``peak_normalizer`` + ``transform_wav`` for a batch
of in-memory songs in one launch; ``load`` adds a stdlib WAV reader for files.

There is no CPU path: waveforms must be on a HIP device (``load`` moves what it reads).
"""
from __future__ import annotations

import math
import wave
from typing import List, Optional

import numpy as np
import torch

from .. import _capi
from .constants import AUDIO_PARAMS
from .sound import chunk_hop


def _hz_to_mel(f: float) -> float:
    return 2595.0 * math.log10(1.0 + f / 700.0)


def melscale_fbanks(n_freqs: int, f_min: float, f_max: float, n_mels: int, sample_rate: int) -> torch.Tensor:
    """torchaudio.functional.melscale_fbanks(..., norm=None, mel_scale="htk") -> [n_freqs, n_mels]
    (float32, computed on the CPU once per Loader: these are plan constants)."""
    all_freqs = torch.linspace(0, sample_rate // 2, n_freqs)
    m_pts = torch.linspace(_hz_to_mel(f_min), _hz_to_mel(f_max), n_mels + 2)
    f_pts = 700.0 * (10.0 ** (m_pts / 2595.0) - 1.0)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts.unsqueeze(0) - all_freqs.unsqueeze(1)
    down = (-1.0 * slopes[:, :-2]) / f_diff[:-1]
    up = slopes[:, 2:] / f_diff[1:]
    return torch.max(torch.zeros(1), torch.min(down, up))


def fbank_bands(fb: torch.Tensor):
    """Dense filterbank [n_freqs, n_mels] -> (lo, n, off, w): each filter's nonzero band is a
    contiguous run of bins (triangles).  A filter with no nonzero bin gets n = 0."""
    n_freqs, n_mels = fb.shape
    lo, n, off, w = [], [], [], []
    pos = 0
    for m in range(n_mels):
        nz = torch.nonzero(fb[:, m] != 0).flatten()
        if nz.numel() == 0:
            lo.append(0), n.append(0), off.append(pos)
            continue
        a, b = int(nz[0]), int(nz[-1]) + 1
        lo.append(a), n.append(b - a), off.append(pos)
        w.append(fb[a:b, m])
        pos += b - a
    wv = torch.cat(w) if w else torch.zeros(1)
    return (torch.tensor(lo, dtype=torch.int32), torch.tensor(n, dtype=torch.int32),
            torch.tensor(off, dtype=torch.int32), wv.to(torch.float32).contiguous())


class Loader:
    """cxai/utils/dataloading.py:13-74 (same constructor) on the HIP front end."""

    def __init__(self, case: Optional[str] = None, sample_rate: int = 16000, n_fft: int = 800, hop_length: int = 360,
                 n_mels: int = 128, slice_length: int = 3, width: int = 128, device=None) -> None:
        if case is not None and case in AUDIO_PARAMS:
            p = AUDIO_PARAMS[case]
            self.sample_rate = p["sample_rate"]
            n_fft, hop_length = p["n_fft"], p["hop_length"]
            self.n_mels = p["n_mels"]
            self.width = p["mel_width"]
            self.slice_length = p.get("slice_length", 0)
            self.num_chunks = p.get("num_chunks", 1)
        else:
            self.sample_rate, self.n_mels, self.slice_length, self.width = sample_rate, n_mels, slice_length, width
            self.num_chunks = 1
        self.n_fft, self.hop_length = n_fft, hop_length
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device()) \
            if torch.cuda.is_available() else None
        self._tables = {}

    # ------------------------------------------------------------------ tables
    def tables(self, device: torch.device):
        key = str(device)
        if key not in self._tables:
            fb = melscale_fbanks(self.n_fft // 2 + 1, 0.0, float(self.sample_rate // 2), self.n_mels,
                                 self.sample_rate)
            lo, n, off, w = fbank_bands(fb)
            self._tables[key] = {
                "window": torch.hann_window(self.n_fft).to(device),
                "lo": lo.to(device), "n": n.to(device), "off": off.to(device), "w": w.to(device),
                "nnz": int(w.numel()), "fb": fb,
            }
        return self._tables[key]

    # --------------------------------------------------------------- transform
    def _run(self, wav: torch.Tensor, n_songs: int, song_stride: int, chunks: int, hop_chunks: int, L: int,
             peak_norm: bool, clamp: bool) -> torch.Tensor:
        _capi.require_gpu(wav, "wav", dtype=torch.float32)
        t = self.tables(wav.device)
        out = torch.empty(n_songs * chunks, 1, self.n_mels, self.width, device=wav.device)
        _capi.call("drsa_amd_logmel", wav.data_ptr(), n_songs, song_stride, chunks, hop_chunks, L, self.n_fft,
                   self.hop_length, self.n_mels, self.width, 1, t["window"].data_ptr(), t["lo"].data_ptr(),
                   t["n"].data_ptr(), t["off"].data_ptr(), t["w"].data_ptr(), t["nnz"], 1 if peak_norm else 0,
                   1 if clamp else 0, -4.0, 1e-7, out.data_ptr(), _capi.stream_ptr(wav.device))
        return out

    def transform_wav(self, wav: torch.Tensor, return_all: bool = False, clamp: bool = True) -> torch.Tensor:
        """dataloading.py:138-176: waveform chunks [..., L] -> log-mel [-1, 1, n_mels, width]
        (frames 1..width of the centred STFT)."""
        if return_all:
            raise NotImplementedError("transform_wav(return_all=True) returns librosa magnitude/phase for plotting "
                                      "(out of scope: presentation code)")
        wav = wav.detach()
        if wav.dtype != torch.float32:
            wav = wav.to(torch.float32)
        wav = wav.contiguous()
        L = wav.size(-1)
        rows = wav.numel() // L if L else 0
        return self._run(wav, rows, L, 1, 0, L, peak_norm=False, clamp=clamp)

    def load_songs(self, songs: torch.Tensor, num_chunks: Optional[int] = None, startpoint: float = 0,
                   peak_norm: bool = True) -> torch.Tensor:
        """Loader.load (dataloading.py:76-111) for songs already in device memory:
        get_slice(slice_length, startpoint, num_chunks) -> peak_normalizer -> transform_wav, one
        launch.  songs [S, T] (or [T]) -> [S*num_chunks, 1, n_mels, width]."""
        if songs.dim() == 1:
            songs = songs[None]
        songs = songs.detach()
        if songs.dtype != torch.float32:
            songs = songs.to(torch.float32)
        songs = songs.contiguous()
        nc = self.num_chunks if num_chunks is None else num_chunks
        S, T = songs.shape
        if self.slice_length == 0:
            return self._run(songs, S, T, 1, 0, T, peak_norm, True)
        L = int(self.slice_length * self.sample_rate)
        if nc > 1:
            hop = chunk_hop(self.slice_length, nc, self.sample_rate)
            usable = min(T, 29 * self.sample_rate)
            n = (usable - L) // hop + 1 if usable >= L else 0
            assert n == nc, "not equal num_chunks"
            return self._run(songs, S, T, nc, hop, L, peak_norm, True)
        start = int(startpoint * self.sample_rate)
        assert startpoint <= T - L, f"Start_point has to be in range [0,{T - L}]"
        return self._run(songs[:, start:].contiguous() if start else songs, S, T - start, 1, 0, L, peak_norm, True)

    def load(self, path_to_audio: str, num_chunks: int = 1, startpoint: int = 0, return_wav: bool = False):
        """dataloading.py:76-111 for a PCM/float WAV file (stdlib reader; torchaudio is not used)."""
        wav = read_wav(path_to_audio)                     # [channels, T] float32 in [-1, 1]
        dev = self.device
        if dev is None:
            raise _capi.DrsaAmdError("Loader.load: no HIP device; drsa_audio_amd has no CPU path")
        wav = wav.to(dev)
        if self.slice_length != 0:
            from .sound import get_slice
            chunks = get_slice(wav, self.slice_length, startpoint, num_chunks, self.sample_rate)
            chunks = chunks.reshape(-1, chunks.size(-1)).contiguous()
            mel = self._run(chunks, chunks.size(0), chunks.size(1), 1, 0, chunks.size(1), True, True)
        else:
            wav = wav.contiguous()
            mel = self._run(wav, wav.size(0), wav.size(1), 1, 0, wav.size(1), True, True)
        if return_wav:
            from .sound import peak_normalizer
            return peak_normalizer(chunks if self.slice_length != 0 else wav), mel
        return mel

    def load_batch(self, songlist: List[str], startpoints: Optional[List[int]] = None) -> torch.Tensor:
        """dataloading.py:113-136."""
        if startpoints is None:
            startpoints = np.zeros(len(songlist))
        samples = [self.load(n, startpoint=s) for n, s in zip(songlist, startpoints)]
        return torch.stack(samples, dim=0).view(-1, 1, self.n_mels, self.width)


def read_wav(path: str) -> torch.Tensor:
    """Minimal RIFF/WAVE reader (8/16/24/32-bit PCM) -> float32 [channels, T] in [-1, 1], the
    scaling of torchaudio.load(normalize=True)."""
    with wave.open(path, "rb") as f:
        ch, sw, n = f.getnchannels(), f.getsampwidth(), f.getnframes()
        raw = f.readframes(n)
    if sw == 1:
        x = (np.frombuffer(raw, np.uint8).astype(np.float32) - 128.0) / 128.0
    elif sw == 2:
        x = np.frombuffer(raw, "<i2").astype(np.float32) / 32768.0
    elif sw == 3:
        b = np.frombuffer(raw, np.uint8).reshape(-1, 3).astype(np.int32)
        v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
        v = np.where(v >= 1 << 23, v - (1 << 24), v)
        x = v.astype(np.float32) / float(1 << 23)
    elif sw == 4:
        x = np.frombuffer(raw, "<i4").astype(np.float32) / float(1 << 31)
    else:
        raise ValueError(f"unsupported sample width {sw}")
    return torch.from_numpy(x.reshape(-1, ch).T.copy())
