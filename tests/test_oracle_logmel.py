"""Log-mel oracle known-answer tests and the front end's host logic (CPU).

torchaudio is absent and no reference file holds a spectrogram, so the oracle is pinned by
known answers (parity vs torchaudio: unpinned; see oracle/logmel_ref.py).
"""
import os
import wave

import numpy as np
import pytest
import torch

import logmel_ref as L


def test_f64_and_torch32_restatements_agree():
    songs = L.synthetic_songs(2, seed=5)
    a = L.load_songs(songs, mode="f64")
    b = L.load_songs(songs, mode="torch32")
    assert a.shape == (16, 1, 128, 128)
    assert np.abs(a - b).max() < 2e-4


def test_toy_case_shapes_and_agreement():
    rng = np.random.default_rng(0)
    wav = rng.standard_normal((3, 16000)).astype(np.float32)
    wav = L.peak_normalizer(wav)
    a = L.transform_wav(wav, "toy", mode="f64")
    b = L.transform_wav(wav, "toy", mode="torch32")
    assert a.shape == (3, 1, 64, 64)
    assert np.abs(a - b).max() < 2e-4


@pytest.mark.parametrize("f0", [220.0, 1000.0, 3100.0, 6500.0])
def test_pure_tone_lands_in_nearest_filter(f0):
    t = np.arange(48000) / 16000
    wav = np.sin(2 * np.pi * f0 * t)[None]
    lm = L.transform_wav(wav, "gtzan", clamp=False)[0, 0]          # [128, 128]
    centres = L.filter_centres(0.0, 8000.0, 128)[1:-1]
    m = int(np.argmax(lm[:, 64]))
    # the tone's bin may straddle two triangles: the winner is one of the two nearest centres
    near = np.argsort(np.abs(centres - f0))[:2]
    assert m in near, (m, near)


def test_filterbank_triangles_peak_at_centres():
    fb = L.melscale_fbanks(401, 0.0, 8000.0, 128, 16000)
    freqs = np.linspace(0, 8000, 401)
    centres = L.filter_centres(0.0, 8000.0, 128)[1:-1]
    for m in range(128):
        col = fb[:, m]
        assert col.max() <= 1.0 + 1e-12 and col.min() >= 0.0
        nz = np.nonzero(col)[0]
        assert np.all(np.diff(nz) == 1), "each triangle is a contiguous band"
        assert abs(freqs[np.argmax(col)] - centres[m]) <= 20.0 + 1e-9     # bin spacing 20 Hz


def test_get_slice_matches_unfold_arithmetic():
    assert L.chunk_hop(3, 8, 16000) == 59200
    song = np.arange(30 * 16000, dtype=np.float64)[None]
    ch = L.get_slice(song, 3, 0, 8, 16000)
    assert ch.shape == (8, 1, 48000)
    assert [int(c[0, 0]) for c in ch] == [i * 59200 for i in range(8)]
    # torch's unfold (the reference's op) agrees
    tch = torch.from_numpy(song)[:, :29 * 16000].unfold(1, 48000, 59200).reshape(-1, 1, 48000)
    assert np.array_equal(tch.numpy(), ch)


def test_product_tables_match_oracle_filterbank():
    from drsa_audio_amd.utils.dataloading import fbank_bands, melscale_fbanks
    for nf, nm in ((401, 128), (241, 64)):
        fb = melscale_fbanks(nf, 0.0, 8000.0, nm, 16000)
        ref = L.melscale_fbanks(nf, 0.0, 8000.0, nm, 16000, mode="torch32")
        assert np.array_equal(fb.numpy(), ref)
        lo, n, off, w = fbank_bands(fb)
        rec = torch.zeros_like(fb)
        for m in range(nm):
            a, k, o = int(lo[m]), int(n[m]), int(off[m])
            rec[a:a + k, m] = w[o:o + k]
        assert torch.equal(rec, fb)


def test_product_slice_helpers_match_oracle():
    from drsa_audio_amd.utils.sound import chunk_hop, get_slice, peak_normalizer
    assert chunk_hop(3, 8, 16000) == L.chunk_hop(3, 8, 16000)
    song = torch.from_numpy(L.synthetic_songs(1, seed=2))
    a = get_slice(song, 3, 0, 8, 16000)
    b = L.get_slice(song.numpy(), 3, 0, 8, 16000)
    assert np.array_equal(a.numpy(), b)
    assert np.array_equal(peak_normalizer(a).numpy(), L.peak_normalizer(b))


@pytest.mark.parametrize("width", [1, 2, 3, 4])
def test_read_wav_roundtrip(tmp_path, width):
    from drsa_audio_amd.utils.dataloading import read_wav
    rng = np.random.default_rng(width)
    x = rng.uniform(-1, 0.99, (2, 1000))
    p = os.path.join(tmp_path, "a.wav")
    if width == 1:
        raw = np.round(x * 128 + 128).clip(0, 255).astype(np.uint8).T.tobytes()
        scale, off = 128.0, 128.0
    else:
        bits = 8 * width
        iv = np.round(x * 2 ** (bits - 1)).astype(np.int64).T
        raw = b"".join(int(v).to_bytes(width, "little", signed=True) for v in iv.flatten())
    with wave.open(p, "wb") as f:
        f.setnchannels(2)
        f.setsampwidth(width)
        f.setframerate(16000)
        f.writeframes(raw)
    y = read_wav(p).numpy()
    assert y.shape == (2, 1000)
    assert np.abs(y - x).max() < 2.0 / 2 ** (8 * width - 1) + 1e-6
