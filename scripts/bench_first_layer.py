"""Micro-benchmark of drsa_amd_first_layer_bwd (pooled) at the bench shape: GTZAN-128 features.0,
B=512 x K=4 clones, 32 channels, 128x128."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from drsa_audio_amd import _capi

dev = torch.device("cuda")
torch.manual_seed(0)
DENSE = os.environ.get("FL_DENSE", "0") == "1"   # VGGish conv0: dense g, B = 32, 64 channels, 128 x 256
if DENSE:
    Bs, clones, C, H, W = 32, 1, 64, 128, 256
else:
    Bs, clones, C, H, W = 512, int(os.environ.get("FL_CLONES", "4")), 32, 128, 128
Bq = Bs * clones
g = torch.randn(Bq, C, H, W, device=dev) if DENSE else torch.randn(Bq, C, H // 2, W // 2, device=dev)
amax = torch.randint(0, 4, (Bs, C, H // 2, W // 2), device=dev, dtype=torch.uint8)
w2 = torch.rand(C, 9, device=dev)
out = torch.empty(Bq, 1, H, W, device=dev)
s = _capi.stream_ptr()


def run():
    _capi.call("drsa_amd_first_layer_bwd", g.data_ptr(), None if DENSE else amax.data_ptr(), w2.data_ptr(), out.data_ptr(), Bq, clones,
               C, H, W, s)


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
byts = g.numel() * 4 + out.numel() * 4 + (0 if DENSE else amax.numel())
oi = out.view(torch.int32).to(torch.int64)
chk = int((oi * (torch.arange(oi.numel(), device=dev, dtype=torch.int64).view_as(oi) % 1000003 + 1)).sum())
print(json.dumps({"lib": os.environ.get("DRSA_AMD_LIB", "default"), "bits_checksum": chk, "ms": ms, "GBs": byts / ms / 1e6, "tflops": 2 * Bq * H * W * C * 9 / ms / 1e9}))
