"""Micro-benchmark of drsa_amd_conv_bwd_first_fused against drsa_amd_conv_bwd + drsa_amd_first_layer_bwd
at the bench shape (GTZAN-128 features.3 -> features.0: B=512 x 4 clones, 32 -> 32 channels, 64x64
cells, pool-sparse g, POST_DIV).  Prints one JSON line of average ms per call."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from drsa_audio_amd import _capi

dev = torch.device("cuda")
S, clones, C, H, W = 512, 4, 32, 64, 64
Bq = S * clones
g = torch.randn(Bq, C, H // 2, W // 2, device=dev)
gam = torch.randint(0, 4, (S, C, H // 2, W // 2), device=dev, dtype=torch.uint8)
wts = torch.randn(_capi.lib().drsa_amd_conv_weight_floats(C, C, 1), device=dev) * 0.1
x = torch.relu(torch.randn(S, C, H, W, device=dev))
den = torch.rand(S, C, H, W, device=dev) + 0.5
am0 = torch.randint(0, 4, (S, C, H, W), device=dev, dtype=torch.uint8)
w2 = torch.rand(C, 9, device=dev)
R = torch.empty(Bq, C, H, W, device=dev)
first = torch.empty(Bq, 1, 2 * H, 2 * W, device=dev)
s = _capi.stream_ptr()


def unfused():
    _capi.call("drsa_amd_conv_bwd", g.data_ptr(), gam.data_ptr(), wts.data_ptr(), x.data_ptr(), den.data_ptr(),
               R.data_ptr(), Bq, clones, C, C, H, W, 1, _capi.XM_MUL, _capi.POST_DIV, 1e-7, s)


def conv_only():
    unfused()


def first_only():
    _capi.call("drsa_amd_first_layer_bwd", R.data_ptr(), am0.data_ptr(), w2.data_ptr(), first.data_ptr(), Bq, clones,
               C, 2 * H, 2 * W, s)


def fused():
    _capi.call("drsa_amd_conv_bwd_first_fused", g.data_ptr(), gam.data_ptr(), wts.data_ptr(), x.data_ptr(),
               den.data_ptr(), None, am0.data_ptr(), w2.data_ptr(), R.data_ptr(), first.data_ptr(), Bq, clones, C, C,
               H, W, 1e-7, s)


def timeit(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / n, 4)


print(json.dumps({"lib": os.environ.get("DRSA_AMD_LIB", "base"), "ff_dbg": os.environ.get("DRSA_AMD_FF_DBG", "0"),
                  "conv_bwd": timeit(conv_only), "first_layer_bwd": timeit(first_only), "fused": timeit(fused)}))
