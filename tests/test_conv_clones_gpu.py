"""Clone-sharing backward conv (csrc/lrp_conv_clones.h) against the per-clone kernel.

drsa_amd_conv_bwd with clones > 1 runs one workgroup per (tile, sample) looping over the K+1
relevance clones; DRSA_AMD_CONV_CLONES=0 selects the per-clone kernel (one workgroup per
(tile, clone)), whose results the exact oracle pins bit for bit (test_lrp_gpu.py,
test_vggish_gpu.py).  Both must agree bit for bit on every rule mode, tile width, ragged
channel count and clone count.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")

# (cin = relevance channels, cout = output channels, H, W, sparse, ng, xmode, post, clones)
CASES = [
    (32, 32, 64, 64, True, 1, 1, 1, 5),     # GTZAN features.3 (Epsilon-type, fused division)
    (64, 32, 32, 32, False, 1, 1, 1, 5),    # features.6
    (64, 64, 16, 16, True, 2, 2, 1, 5),     # Gamma split, W = 16 tiles
    (64, 64, 8, 8, False, 2, 2, 2, 3),      # W = 8 tiles, ReLU mask
    (128, 64, 16, 16, True, 1, 0, 0, 2),    # plain gradient
    (32, 20, 32, 32, True, 1, 1, 1, 4),     # ragged output channels
    (20, 32, 24, 36, False, 1, 1, 2, 33),   # ragged input channels, partial tiles, K = 32
    (64, 32, 32, 32, True, 2, 1, 1, 9),     # two weight sets with the MUL mode (second set unused)
]


def _pad32(c):
    return (c + 31) // 32 * 32


def _run(case, use_clones, seed=0):
    from drsa_audio_amd import _capi
    cin, cout, H, W, sparse, ng, xmode, post, clones = case
    torch.manual_seed(seed)
    Bs = 3
    Bq = Bs * clones
    if sparse:
        g = torch.randn(Bq, cin, H // 2, W // 2, device=DEV)
        amax = torch.randint(0, 4, (Bs, cin, H // 2, W // 2), device=DEV, dtype=torch.uint8)
    else:
        g = torch.randn(Bq, cin, H, W, device=DEV)
        amax = None
    w = torch.randn(ng, 9 * _pad32(cin), _pad32(cout), device=DEV)
    x = torch.randn(Bs, cout, H, W, device=DEV)
    den = torch.randn(Bs, cout, H, W, device=DEV)
    den[0, 0, :2] = 0.0                      # stabiliser path
    out = torch.full((Bq, cout, H, W), float("nan"), device=DEV)
    old = os.environ.get("DRSA_AMD_CONV_CLONES")
    os.environ["DRSA_AMD_CONV_CLONES"] = "1" if use_clones else "0"
    try:
        _capi.call("drsa_amd_conv_bwd", g.data_ptr(), amax.data_ptr() if amax is not None else None,
                   w.data_ptr(), x.data_ptr(), den.data_ptr(), out.data_ptr(), Bq, clones, cin, cout, H, W,
                   ng, xmode, post, 1e-6, _capi.stream_ptr())
        torch.cuda.synchronize()
    finally:
        if old is None:
            os.environ.pop("DRSA_AMD_CONV_CLONES")
        else:
            os.environ["DRSA_AMD_CONV_CLONES"] = old
    return out.cpu()


@pytest.mark.parametrize("case", CASES, ids=[f"c{i}" for i in range(len(CASES))])
def test_clone_kernel_equals_per_clone_kernel(case):
    a = _run(case, True)
    b = _run(case, False)
    assert not torch.isnan(a).any(), "clone kernel left outputs unwritten"
    assert torch.equal(a.view(torch.int32), b.view(torch.int32))


def test_clone_kernel_writes_nothing_outside_the_batch():
    """Guard rows around the output: the out-of-range buffer stores must be dropped."""
    from drsa_audio_amd import _capi
    cin, cout, H, W, clones, Bs = 32, 32, 64, 64, 5, 2
    g = torch.randn(Bs * clones, cin, H // 2, W // 2, device=DEV)
    amax = torch.randint(0, 4, (Bs, cin, H // 2, W // 2), device=DEV, dtype=torch.uint8)
    w = torch.randn(1, 9 * cin, cout, device=DEV)
    x = torch.randn(Bs, cout, H, W, device=DEV)
    den = torch.randn(Bs, cout, H, W, device=DEV)
    buf = torch.full((Bs * clones + 2, cout, H, W), 7.0, device=DEV)
    out = buf[1:-1]
    _capi.call("drsa_amd_conv_bwd", g.data_ptr(), amax.data_ptr(), w.data_ptr(), x.data_ptr(), den.data_ptr(),
               out.data_ptr(), Bs * clones, clones, cin, cout, H, W, 1, 1, 1, 1e-6, _capi.stream_ptr())
    torch.cuda.synchronize()
    assert torch.all(buf[0] == 7.0) and torch.all(buf[-1] == 7.0)
    assert not torch.any(out == 7.0)
