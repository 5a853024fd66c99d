"""Polar (Newton-Schulz) iteration counts and timing at d = 64 / 128 for DRSA-like V = U + G."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from drsa_audio_amd import _capi

dev = torch.device("cuda")
out = {}
for d in (64, 128):
    rng = np.random.default_rng(d)
    U = np.linalg.qr(rng.standard_normal((d, d)))[0]
    for scale in (1e-3, 1e-2, 1e-1):
        V = torch.from_numpy((U + scale * rng.standard_normal((d, d))).astype(np.float32)).to(dev)
        Uo = torch.empty_like(V)
        it = torch.zeros(1, dtype=torch.int32, device=dev)
        s = _capi.stream_ptr()
        for _ in range(3):
            _capi.call("drsa_amd_polar", V.data_ptr(), d, Uo.data_ptr(), it.data_ptr(), s)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            _capi.call("drsa_amd_polar", V.data_ptr(), d, Uo.data_ptr(), it.data_ptr(), s)
        e1.record()
        torch.cuda.synchronize()
        Un = Uo.cpu().double().numpy()
        u, _, vt = np.linalg.svd(V.cpu().double().numpy())
        out[f"d{d}_s{scale}"] = {"iters": int(it.item()), "ms": e0.elapsed_time(e1) / 20,
                                 "err_vs_svd": float(np.abs(Un - u @ vt).max())}
print(json.dumps(out, indent=1))
