"""Micro-benchmark of the Cin = 1 forward (csrc/conv_first.hip) at the bench shape: GTZAN-128
features.0, B=512, 32 channels, 128x128, WSquare den map; sweeps DRSA_AMD_FIRST_FWD_CSPLIT."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from drsa_audio_amd import _capi

dev = torch.device("cuda")
B, C, H, W = 512, 32, 128, 128
x = torch.randn(B, 1, H, W, device=dev)
wts = torch.randn(1, 9, C, device=dev)
bias = torch.randn(3, C, device=dev)
den_map = torch.rand(C, H, W, device=dev)
out = torch.empty(B, C, H // 2, W // 2, device=dev)
amax = torch.empty(B, C, H // 2, W // 2, device=dev, dtype=torch.uint8)
den = torch.empty_like(out)
s = _capi.stream_ptr()


NODEN = os.environ.get("NODEN") == "1"
RING = os.environ.get("RING", "1") == "1"   # the engine's form: den copy on the border ring only
den_ring = torch.empty(B, C, 2 * (W // 2) + 8 * (H // 2 - 2), device=dev)


def run():
    if RING and not NODEN:
        _capi.call("drsa_amd_conv_fwd_den_ring", x.data_ptr(), wts.data_ptr(), bias.data_ptr(), den_map.data_ptr(),
                   out.data_ptr(), amax.data_ptr(), den_ring.data_ptr(), B, C, H, W, 1, s)
        return
    _capi.call("drsa_amd_conv_fwd", x.data_ptr(), wts.data_ptr(), bias.data_ptr(), None if NODEN else den_map.data_ptr(),
               out.data_ptr(), amax.data_ptr(), None if NODEN else den.data_ptr(), B, 1, C, H, W, 1, 1, s)


for cs in sys.argv[1:] or ["0"]:
    os.environ["DRSA_AMD_FIRST_FWD_CSPLIT"] = cs
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
    byts = x.numel() * 4 + out.numel() * 9
    print(json.dumps({"lib": os.environ.get("DRSA_AMD_LIB", "base"), "noden": NODEN, "ring": RING, "csplit": cs,
                      "ms": ms, "GBs": byts / ms / 1e6}))
