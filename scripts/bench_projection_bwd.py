"""Micro-benchmark of drsa_amd_projection_bwd at the bench shape (GTZAN-128 j=7: B=512, d=64,
32x32 maps, K=4, 2x2 pool after, K+1 fan-out)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from drsa_audio_amd import _capi

dev = torch.device("cuda")
torch.manual_seed(0)
B, D, H, W, K = 512, 64, 32, 32, 4
g = torch.randn(B, D, H // 2, W // 2, device=dev)
amax = torch.randint(0, 4, (B, D, H // 2, W // 2), device=dev, dtype=torch.uint8)
ap, h, a = (torch.randn(B, D, H, W, device=dev) for _ in range(3))
den = torch.rand(B, D, H, W, device=dev) + 0.5
U = torch.from_numpy(np.linalg.qr(np.random.default_rng(0).standard_normal((D, D)))[0].astype(np.float32)).to(dev)
G = torch.empty(B * (K + 1), D, H, W, device=dev)
s = _capi.stream_ptr()
P = torch.empty_like(U)
_capi.call("drsa_amd_projection_residual", U.data_ptr(), D, P.data_ptr(), s)


RC = os.environ.get("RC", "1") == "1"   # recompute h and a' (engine default) vs stored buffers
FAN = int(os.environ.get("FAN", "2"))   # 2: K concept clones (the engine default since round 3); 1: K+1


def run():
    _capi.call("drsa_amd_projection_bwd", g.data_ptr(), amax.data_ptr(), None if RC else ap.data_ptr(),
               None if RC else h.data_ptr(), a.data_ptr(),
               den.data_ptr(), U.data_ptr(), P.data_ptr(), G.data_ptr(), B, D, H, W, K, 1e-6, 1e-7, FAN, s)


for _ in range(3):
    run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    run()
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 20
byts = (g.numel() + 4 * a.numel() + G.numel()) * 4 + amax.numel()
nq = K if FAN == 2 else K + 1
Gi = G[:B * nq].view(torch.int32).to(torch.int64)
chk = int((Gi * (torch.arange(Gi.numel(), device=dev, dtype=torch.int64).view_as(Gi) % 1000003 + 1)).sum())
print(json.dumps({"lib": os.environ.get("DRSA_AMD_LIB", "default"), "rc": RC, "ms": ms, "bits_checksum": chk, "GBs": byts / ms / 1e6, "tflops": 2 * 3 * B * H * W * D * D / ms / 1e9}))
