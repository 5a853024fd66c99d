"""4 x 8-tile conv kernels (conv_small.hip) against the 8 x 8 kernels they replace.

lrp_conv.hip's launch() swaps a 4 x 8-tile kernel in for an 8 x 8 entry when the 8 x 8 grid would
have fewer than 512 workgroups, so which kernel a layer runs depends on the batch.  Both keep every
output one k-ordered fp32 chain (k = ci * 9 + tap), so a sample's outputs must not depend on the
batch it is run in: each case runs the same leading samples once in a batch below the threshold
(4 x 8 tiles) and once in a batch at the threshold (8 x 8 tiles) and asserts bit equality, for every
replaced family: forwards with 2 x 2 pool or ReLU only, NG 1-3 (with the denominator output), and
backwards with dense and pool-sparse g, NG 1 / 2, no post, POST_DIV and POST_MASK, 1 and 2 clones."""
import pytest
import torch

from drsa_audio_amd import _capi

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
SMALL_WG = 512          # lrp_conv.hip DRSA_CONV_SMALL_WG


def _batches(H, W):
    tiles = ((H + 7) // 8) * ((W + 7) // 8)
    return 4, SMALL_WG // tiles            # 4 x 8 tiles below, 8 x 8 tiles at the threshold


def _rep(t, n):
    reps = (n + t.size(0) - 1) // t.size(0)
    return t.repeat(reps, *([1] * (t.dim() - 1)))[:n].contiguous()


@pytest.mark.parametrize("cin,cout", [(64, 128), (128, 128)])
@pytest.mark.parametrize("HW", [8, 16])
@pytest.mark.parametrize("ng", [1, 2, 3])
@pytest.mark.parametrize("pool", [0, 1])
def test_small_forward_equals_8x8(cin, cout, HW, ng, pool):
    lib = _capi.lib()
    H = W = HW
    bs, bb = _batches(H, W)
    g = torch.Generator().manual_seed(cin + HW + 10 * ng + pool)
    x = torch.randn(bs, cin, H, W, generator=g)
    if ng == 2:
        x = x.abs()                                   # NG = 2 is the Gamma forward on x >= 0 (ABI)
    n = lib.drsa_amd_conv_weight_floats(cin, cout, ng)
    wts = (torch.randn(n, generator=g) * 0.05).to(DEV)
    b3 = (torch.randn(3, cout, generator=g) * 0.1).to(DEV)
    s = _capi.stream_ptr(DEV)
    outs = []
    for B in (bs, bb):
        xb = _rep(x, B).to(DEV)
        Ho, Wo = (H // 2, W // 2) if pool else (H, W)
        y = torch.full((B, cout, Ho, Wo), float("nan"), device=DEV)
        am = torch.zeros(B, cout, Ho, Wo, dtype=torch.uint8, device=DEV) if pool else None
        den = torch.full((B, cout, Ho, Wo), float("nan"), device=DEV)
        _capi.call("drsa_amd_conv_fwd", xb.data_ptr(), wts.data_ptr(), b3.data_ptr(), None, y.data_ptr(),
                   _capi.ptr(am), den.data_ptr(), B, cin, cout, H, W, ng, pool, s)
        outs.append((y, am, den))
    torch.cuda.synchronize()
    (y0, a0, d0), (y1, a1, d1) = outs
    assert not torch.isnan(y0).any() and not torch.isnan(d0).any()
    assert torch.equal(y0, y1[:bs]) and torch.equal(d0, d1[:bs])
    if pool:
        assert torch.equal(a0, a1[:bs])


@pytest.mark.parametrize("cin,cout", [(128, 64), (128, 128)])
@pytest.mark.parametrize("HW", [8, 16])
@pytest.mark.parametrize("sparse", [False, True])
@pytest.mark.parametrize("ng,post,clones", [(1, _capi.POST_NONE, 1), (1, _capi.POST_DIV, 2), (2, _capi.POST_DIV, 1),
                                            (1, _capi.POST_MASK, 1)])
def test_small_backward_equals_8x8(cin, cout, HW, sparse, ng, post, clones):
    lib = _capi.lib()
    H = W = HW
    bs, bb = _batches(H, W)
    g = torch.Generator().manual_seed(cin + HW + 3 * ng + 7 * post + sparse)
    S = bs // clones
    xmode = _capi.XM_SPLIT if ng == 2 else _capi.XM_MUL
    x = torch.randn(S, cout, H, W, generator=g)       # signed: the x+ / x- split of NG = 2
    den = torch.randn(S, cout, H, W, generator=g)
    if sparse:
        gin = torch.randn(bs, cin, H // 2, W // 2, generator=g)
        gam = torch.randint(0, 4, (S, cin, H // 2, W // 2), generator=g, dtype=torch.uint8)
    else:
        gin = torch.randn(bs, cin, H, W, generator=g)
        gam = None
    n = lib.drsa_amd_conv_weight_floats(cin, cout, ng)
    wts = (torch.randn(n, generator=g) * 0.05).to(DEV)
    s = _capi.stream_ptr(DEV)
    outs = []
    for B in (bs, bb):
        Sb = B // clones
        xb, db = _rep(x, Sb).to(DEV), _rep(den, Sb).to(DEV)
        gb = _rep(gin, B).to(DEV)
        ab = _rep(gam, Sb).to(DEV) if sparse else None
        o = torch.full((B, cout, H, W), float("nan"), device=DEV)
        _capi.call("drsa_amd_conv_bwd", gb.data_ptr(), _capi.ptr(ab), wts.data_ptr(), xb.data_ptr(),
                   db.data_ptr() if post == _capi.POST_DIV else None, o.data_ptr(), B, clones, cin, cout, H, W, ng,
                   xmode, post, 1e-6, s)
        outs.append(o)
    torch.cuda.synchronize()
    assert not torch.isnan(outs[0]).any()
    assert torch.equal(outs[0], outs[1][:bs])
