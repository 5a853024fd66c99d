"""Micro-benchmark of drsa_amd_projection_fwd at the bench shape (GTZAN-128 j=7: B=512, d=64,
32x32, pooled).  DRSA_AMD_PROJ_PLDS=0 / 1 picks where the residual P lives."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from drsa_audio_amd import _capi

B, D, H, W = 512, 64, 32, 32
dev = torch.device("cuda")
a = torch.relu(torch.randn(B, D, H, W, device=dev))
U = torch.from_numpy(np.linalg.qr(np.random.default_rng(0).standard_normal((D, D)))[0].astype(np.float32)).to(dev)
P = torch.empty_like(U)
s = _capi.stream_ptr()
_capi.call("drsa_amd_projection_residual", U.data_ptr(), D, P.data_ptr(), s)
y = torch.empty(B, D, H // 2, W // 2, device=dev)
amax = torch.empty(B, D, H // 2, W // 2, device=dev, dtype=torch.uint8)


def run():
    _capi.call("drsa_amd_projection_fwd", a.data_ptr(), U.data_ptr(), P.data_ptr(), None, None, y.data_ptr(),
               amax.data_ptr(), B, D, H, W, 1, s)


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
print(json.dumps({"plds": os.environ.get("DRSA_AMD_PROJ_PLDS", "default"), "ms": ms,
                  "tflops": 2 * 2 * B * H * W * D * D / (ms * 1e-3) / 1e12}))
