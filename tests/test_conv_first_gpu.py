"""First-layer forward (Cin = 1, fused ReLU + 2x2 pool + argmax + den; csrc/conv_first.hip)
vs the exact-order oracle, called through the C ABI (GPU).

Parity: y, argmax and den are bit-identical to oracle/lrp_exact.c:conv2d_exact per weight set
followed by torch's relu / max_pool2d(return_indices) and the rule denominators of SURVEY
App. A (WSquare map, Epsilon z + b, Gamma (z+ + b+) + (z- + b-)).  Inputs include negative
values (log-mel), exact ties (zero rows -> relu plateaus) and a NaN.
"""
import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

import lrp_ref
from drsa_audio_amd import _capi

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _exact_conv(x, w, b):
    m = nn.Conv2d(1, w.size(0), 3, padding=1)
    return lrp_ref.ExactOps.conv(m, x, w, b)


def _pool(y):
    B, C, H, W = y.shape
    win = y.reshape(B, C, H // 2, 2, W // 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(B, C, H // 2, W // 2, 4)
    m, am = win[..., 0].clone(), torch.zeros(win.shape[:-1], dtype=torch.uint8)
    for s in range(1, 4):
        v = win[..., s]
        take = (v > m) | (torch.isnan(v) & ~torch.isnan(m))
        m = torch.where(take, v, m)
        am = torch.where(take, torch.full_like(am, s), am)
    return m, am


def _at_argmax(full, am):
    B, C, H, W = full.shape
    win = full.reshape(B, C, H // 2, 2, W // 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(B, C, H // 2, W // 2, 4)
    return torch.gather(win, -1, am.long().unsqueeze(-1)).squeeze(-1)


@pytest.mark.parametrize("ng,den", [(1, "none"), (1, "map"), (1, "map_unaligned"), (1, "eps"), (2, "gamma"),
                                    (3, "gamma")])
@pytest.mark.parametrize("shape", [(3, 32, 16, 24), (2, 64, 128, 128), (1, 32, 8, 8)])
def test_first_conv_pool_bit_exact(ng, den, shape):
    B, cout, H, W = shape
    g = torch.Generator().manual_seed(ng * 100 + H)
    x = torch.randn(B, 1, H, W, generator=g) * 3.0
    if ng == 2:
        x = x.abs()                       # ng = 2 is the Gamma forward on x >= 0 (ABI contract)
    x[0, 0, 2:4, :] = 0.0                 # ties: relu plateau inside windows
    if B > 1 and den != "gamma":          # (the Gamma split of a NaN input is not pinned)
        x[1, 0, 5, 7] = float("nan")
    w = torch.randn(cout, 1, 3, 3, generator=g)
    bias = torch.randn(cout, generator=g) * 0.1
    cout_p = (cout + 31) // 32 * 32
    sets = [w, w.clamp(min=0), w.clamp(max=0)][:ng]
    bsets = [bias, bias.clamp(min=0), bias.clamp(max=0)]
    if den == "eps":
        bsets[1] = bias * 0.5
    wdev = torch.zeros(ng, 9, cout_p)
    for s, ws in enumerate(sets):
        wdev[s, :, :cout] = ws.reshape(cout, 9).T
    bdev = torch.zeros(3, cout_p)
    for s in range(3):
        bdev[s, :cout] = bsets[s]

    z = _exact_conv(x, w, bias)
    y = torch.where(torch.isnan(z), z, z.clamp(min=0))
    y_ref, am_ref = _pool(y)
    den_map = None
    if den.startswith("map"):
        den_map = torch.rand(cout, H, W, generator=g) + 0.5
        den_full = den_map.unsqueeze(0).expand(B, -1, -1, -1).contiguous()
    elif den == "eps":
        den_full = _exact_conv(x, w, None) + bsets[1].view(1, -1, 1, 1)
    elif den == "gamma":
        zp = _exact_conv(x.clamp(min=0), sets[1], None) + bsets[1].view(1, -1, 1, 1)
        zn = (_exact_conv(x.clamp(max=0), sets[2], None) if ng == 3 else torch.zeros_like(zp)) \
            + bsets[2].view(1, -1, 1, 1)
        den_full = zp + zn
    xd = x.to(DEV).contiguous()
    out = torch.full((B, cout, H // 2, W // 2), -7.0, device=DEV)
    amax = torch.full((B, cout, H // 2, W // 2), 9, dtype=torch.uint8, device=DEV)
    out_den = torch.full_like(out, -7.0) if den != "none" else None
    # keep every device operand referenced until the kernel has run
    wd, bd = wdev.to(DEV), bdev.to(DEV)
    dm = None if den_map is None else den_map.to(DEV).contiguous()
    if den == "map_unaligned":            # a map pointer off the 16-byte grid (the map is gathered per pixel)
        dm = torch.cat([torch.zeros(1), den_map.flatten()]).to(DEV)[1:]
        assert dm.data_ptr() % 16 != 0
    _capi.call("drsa_amd_conv_fwd", xd.data_ptr(), wd.data_ptr(), bd.data_ptr(), _capi.ptr(dm), out.data_ptr(),
               amax.data_ptr(), _capi.ptr(out_den), B, 1, cout, H, W, ng, 1, _capi.stream_ptr(DEV))
    torch.cuda.synchronize()
    bad = (amax.cpu() != am_ref).nonzero()
    assert bad.numel() == 0, (f"{bad.size(0)} argmax mismatches, first {bad[:4].tolist()}: "
                              f"got {amax.cpu()[tuple(bad[0])]} want {am_ref[tuple(bad[0])]}; "
                              f"y got {out.cpu()[tuple(bad[0])]} want {y_ref[tuple(bad[0])]}")
    o = out.cpu()
    assert torch.equal(torch.isnan(o), torch.isnan(y_ref))
    assert torch.equal(torch.nan_to_num(o, nan=0.0), torch.nan_to_num(y_ref, nan=0.0))
    if out_den is not None:
        d_ref = _at_argmax(den_full, am_ref)
        d = out_den.cpu()
        assert torch.equal(torch.isnan(d), torch.isnan(d_ref))
        assert torch.equal(torch.nan_to_num(d, nan=0.0), torch.nan_to_num(d_ref, nan=0.0))
