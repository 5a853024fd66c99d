"""WSquare / Flat first layer with its denominator in ring form (GPU, through the C ABI):
drsa_amd_conv_fwd_den_ring stores the per-sample copy at the pool argmax only on the image's border
ring of float4 groups (compactly), and drsa_amd_conv_bwd_den_ring divides by it there and by the
map's per-channel interior value elsewhere.

Parity: bit-identical to drsa_amd_conv_fwd (map den, 2x2 pool) + drsa_amd_conv_bwd(POST_DIV) on
the full copy, for fp32 and bf16 backward weights, dense and pool-sparse g, Epsilon-type (XM_MUL)
and plain (XM_NONE) rules, clones > 1 -- with the copy's interior filled with NaN, so a read of a
value the ring forward did not store would show; plus the engine at plan level (GTZAN standard
LRP and HeatmapGenerator) against the per-sample copy (plan._DEN_COPY)."""
import numpy as np
import pytest
import torch

from drsa_audio_amd import _capi

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _first_layer(S, C, H2, W2, seed):
    """Input, WSquare map (drsa_amd_first_layer_den) and the first layer's forward both ways."""
    g = torch.Generator().manual_seed(seed)
    H, W = 2 * H2, 2 * W2
    x = (torch.randn(S, 1, H, W, generator=g) * 2).to(DEV)
    w = torch.randn(C, 1, 3, 3, generator=g)
    b = torch.randn(C, generator=g) * 0.1
    cp = (C + 31) // 32 * 32
    wts = torch.zeros(1, 9, cp)
    wts[0, :, :C] = w.reshape(C, 9).T
    b3 = torch.zeros(3, cp)
    b3[0, :C] = b
    wts, b3 = wts.to(DEV).contiguous(), b3.to(DEV).contiguous()
    w2 = (w ** 2).to(DEV).contiguous()
    bb2 = (b ** 2).to(DEV).contiguous()
    dmap = torch.empty(C, H, W, device=DEV)
    s = _capi.stream_ptr(DEV)
    _capi.call("drsa_amd_first_layer_den", w2.data_ptr(), bb2.data_ptr(), dmap.data_ptr(), C, 1, H, W, s)
    outs = {}
    for ring in (False, True):
        y = torch.empty(S, C, H2, W2, device=DEV)
        am = torch.empty(S, C, H2, W2, dtype=torch.uint8, device=DEV)
        if ring:
            den = torch.full((S, C, 2 * W2 + 8 * (H2 - 2)), float("nan"), device=DEV)
            _capi.call("drsa_amd_conv_fwd_den_ring", x.data_ptr(), wts.data_ptr(), b3.data_ptr(), dmap.data_ptr(),
                       y.data_ptr(), am.data_ptr(), den.data_ptr(), S, C, H, W, 1, s)
        else:
            den = torch.full((S, C, H2, W2), float("nan"), device=DEV)
            _capi.call("drsa_amd_conv_fwd", x.data_ptr(), wts.data_ptr(), b3.data_ptr(), dmap.data_ptr(),
                       y.data_ptr(), am.data_ptr(), den.data_ptr(), S, 1, C, H, W, 1, 1, s)
        outs[ring] = (y, am, den)
    torch.cuda.synchronize()
    c4 = dmap[:, 1, 1].reshape(-1, 1).expand(-1, 4).contiguous()
    return dmap, c4, outs


@pytest.mark.parametrize("C,H2,W2", [(32, 64, 64), (32, 8, 16), (16, 6, 8), (8, 2, 8), (64, 8, 16), (40, 4, 8)])
def test_first_layer_ring_forward_and_map_interior(C, H2, W2):
    dmap, c4, outs = _first_layer(3, C, H2, W2, seed=C + H2)
    inner = dmap[:, 1:-1, 1:-1]
    assert torch.equal(inner, dmap[:, 1:2, 1:2].expand_as(inner))      # the property the ring form uses
    (y0, a0, d0), (y1, a1, d1) = outs[False], outs[True]
    assert torch.equal(y0, y1) and torch.equal(a0, a1)
    ring = torch.zeros(H2, W2, dtype=torch.bool, device=DEV)
    ring[0, :] = ring[-1, :] = True
    ring[:, :4] = ring[:, -4:] = True
    # the compact ring, expanded: row 0, row H2-1, then rows 1..H2-2 x (4 + 4 columns)
    full = torch.full_like(d0, float("nan"))
    full[..., 0, :] = d1[..., :W2]
    full[..., -1, :] = d1[..., W2:2 * W2]
    side = d1[..., 2 * W2:].reshape(d1.size(0), C, H2 - 2, 8)
    full[..., 1:-1, :4] = side[..., :4]
    full[..., 1:-1, -4:] = side[..., 4:]
    assert not torch.isnan(d1).any()                                    # every ring slot is stored
    assert torch.equal(full[..., ring], d0[..., ring])
    # off the ring the full copy equals the per-channel interior value
    assert torch.equal(d0[..., ~ring], c4[:, :1].reshape(1, C, 1).expand(d0.size(0), C, int((~ring).sum())))


@pytest.mark.parametrize("cin,H2,W2", [(32, 64, 64), (64, 32, 32), (32, 16, 16), (64, 8, 8)])
@pytest.mark.parametrize("sparse", [True, False])
@pytest.mark.parametrize("bf16", [False, True])
@pytest.mark.parametrize("xmode", [_capi.XM_MUL, _capi.XM_NONE])
def test_conv_bwd_den_ring_equals_post_div_on_full_copy(cin, H2, W2, sparse, bf16, xmode):
    lib = _capi.lib()
    cout = 32
    if bf16 and not lib.drsa_amd_conv_bwd_has_kernel_bf16(cin, cout, W2, 1, int(sparse)):
        pytest.skip("no bf16 kernel for this shape")
    S, clones = 3, 2
    Bq = S * clones
    dmap, c4, outs = _first_layer(S, cout, H2, W2, seed=cin + H2 + 7 * sparse)
    y, am, d_full = outs[False]
    _, _, d_ring = outs[True]
    g = torch.Generator().manual_seed(cin * 3 + H2)
    if sparse:
        gin = torch.randn(Bq, cin, H2 // 2, W2 // 2, generator=g).to(DEV)
        gam = torch.randint(0, 4, (S, cin, H2 // 2, W2 // 2), generator=g, dtype=torch.uint8).to(DEV)
    else:
        gin = torch.randn(Bq, cin, H2, W2, generator=g).to(DEV)
        gam = None
    if bf16:
        n = lib.drsa_amd_conv_weight_bf16_elems(cin, cout, 1)
        wts = (torch.randn(n, generator=g) * 0.1).to(torch.bfloat16).view(torch.int16).to(DEV)
    else:
        n = lib.drsa_amd_conv_weight_floats(cin, cout, 1)
        wts = (torch.randn(n, generator=g) * 0.1).to(DEV)
    o_ref = torch.full((Bq, cout, H2, W2), -9.0, device=DEV)
    o_r = torch.full_like(o_ref, -7.0)
    s = _capi.stream_ptr(DEV)
    eps = 1e-7
    fn = "drsa_amd_conv_bwd_bf16" if bf16 else "drsa_amd_conv_bwd"
    _capi.call(fn, gin.data_ptr(), _capi.ptr(gam), wts.data_ptr(), y.data_ptr(), d_full.data_ptr(), o_ref.data_ptr(),
               Bq, clones, cin, cout, H2, W2, 1, xmode, _capi.POST_DIV, eps, s)
    _capi.call("drsa_amd_conv_bwd_den_ring", gin.data_ptr(), _capi.ptr(gam), wts.data_ptr(), int(bf16), y.data_ptr(),
               d_ring.data_ptr(), c4.data_ptr(), o_r.data_ptr(), Bq, clones, cin, cout, H2, W2, 1, xmode, eps, s)
    torch.cuda.synchronize()
    assert not torch.isnan(o_r).any()
    assert torch.equal(o_r, o_ref)


def test_ring_entries_reject_missing_operands():
    lib = _capi.lib()
    assert lib.drsa_amd_conv_bwd_den_ring(None, None, None, 0, None, None, None, None, 2, 1, 32, 32, 8, 8, 1, 1,
                                          0.0, None) == -1
    assert lib.drsa_amd_conv_fwd_den_ring(None, None, None, None, None, None, None, 1, 32, 8, 8, 1, None) == -1


@pytest.mark.parametrize("hg", [False, True])
def test_plan_ring_equals_den_copy(monkeypatch, hg):
    """The engine with the ring form (default) and with the full copy (plan._DEN_COPY) gives
    identical relevances / heatmaps (GTZAN: WSquare first layer, 2x2 pool)."""
    import copy
    import drsa_audio_amd.engine.plan as plan
    from drsa_audio_amd.engine import clear_cache
    from drsa_audio_amd.utils.constants import LRP_NAME_MAP_GTZAN
    from drsa_audio_amd.xai.explain.attribute import compute_relevances
    from drsa_audio_amd.xai.explain.explainer import HeatmapGenerator
    from drsa_audio_amd.zennit.composites import NameMapComposite
    from lrp_common import gtzan128, logmel, u64
    net = gtzan128().to(DEV)
    x = logmel(6, seed=17).to(DEV)
    outs = []
    for copy_den in (False, True):
        monkeypatch.setattr(plan, "_DEN_COPY", copy_den)
        clear_cache()
        if hg:
            h = HeatmapGenerator(copy.deepcopy(net), u64(), LRP_NAME_MAP_GTZAN, "rock", num_concepts=4, layer_idx=7,
                                 device=DEV, standard="sum")
            h.generate_subspace_heatmaps(x)
            outs.append({k: h.info[k] for k in ("standard_heatmaps", "subspace_heatmaps", "mask")})
        else:
            R = compute_relevances(net, x, NameMapComposite(LRP_NAME_MAP_GTZAN), class_idx=2)
            outs.append({"R": R.cpu().numpy()})
    clear_cache()
    for k in outs[0]:
        assert np.array_equal(outs[0][k], outs[1][k]), k


@pytest.mark.parametrize("cin,H,W,sparse,bf16,pool_w", [(64, 16, 256, False, False, 2), (64, 16, 32, True, False, 2),
                                                        (64, 16, 256, True, True, 4), (64, 16, 64, False, True, 2),
                                                        (64, 8, 16, True, True, 2)])
def test_conv_bwd_den_map_equals_post_div_on_copy(cin, H, W, sparse, bf16, pool_w):
    """drsa_amd_conv_bwd_den_map (the next layer's denominator = its map, one plane for every
    sample: a WSquare layer without a pool, VGGish conv0 -> conv3) equals POST_DIV on the
    per-sample copy, bit for bit."""
    lib = _capi.lib()
    cout, S, clones = 64, 3, 2
    Bq = S * clones
    g = torch.Generator().manual_seed(cin + W + pool_w)
    if sparse:
        gin = torch.randn(Bq, cin, H // 2, W // pool_w, generator=g).to(DEV)
        gam = torch.randint(0, 2 * pool_w, (S, cin, H // 2, W // pool_w), generator=g, dtype=torch.uint8).to(DEV)
    else:
        gin = torch.randn(Bq, cin, H, W, generator=g).to(DEV)
        gam = None
    x = (torch.randn(S, cout, H, W, generator=g).abs() * (torch.rand(S, cout, H, W, generator=g) > 0.3)).to(DEV)
    dmap = torch.randn(cout, H, W, generator=g).to(DEV)
    dcopy = dmap.unsqueeze(0).expand(S, -1, -1, -1).contiguous()
    if bf16:
        n = lib.drsa_amd_conv_weight_bf16_elems(cin, cout, 1)
        wts = (torch.randn(n, generator=g) * 0.1).to(torch.bfloat16).view(torch.int16).to(DEV)
    else:
        n = lib.drsa_amd_conv_weight_floats(cin, cout, 1)
        wts = (torch.randn(n, generator=g) * 0.1).to(DEV)
    o_ref = torch.full((Bq, cout, H, W), -9.0, device=DEV)
    o_m = torch.full_like(o_ref, -7.0)
    s = _capi.stream_ptr(DEV)
    if bf16 and sparse and pool_w == 4:
        _capi.call("drsa_amd_conv_bwd_bf16_pw", gin.data_ptr(), gam.data_ptr(), 4, wts.data_ptr(), x.data_ptr(),
                   dcopy.data_ptr(), o_ref.data_ptr(), Bq, clones, cin, cout, H, W, _capi.XM_MUL, _capi.POST_DIV, 1e-7, s)
    else:
        fn = "drsa_amd_conv_bwd_bf16" if bf16 else "drsa_amd_conv_bwd"
        _capi.call(fn, gin.data_ptr(), _capi.ptr(gam), wts.data_ptr(), x.data_ptr(), dcopy.data_ptr(), o_ref.data_ptr(),
                   Bq, clones, cin, cout, H, W, 1, _capi.XM_MUL, _capi.POST_DIV, 1e-7, s)
    _capi.call("drsa_amd_conv_bwd_den_map", gin.data_ptr(), _capi.ptr(gam), pool_w, wts.data_ptr(), int(bf16),
               x.data_ptr(), dmap.data_ptr(), o_m.data_ptr(), Bq, clones, cin, cout, H, W, 1, _capi.XM_MUL, 1e-7, s)
    torch.cuda.synchronize()
    assert torch.equal(o_m, o_ref)


@pytest.mark.parametrize("bf16_bwd", [False, True])
def test_vggish_plan_den_map_equals_den_copy(monkeypatch, bf16_bwd):
    """VGGish-BN (WSquare conv0 -> conv3, no pool between): the plan reading the map itself equals
    the plan with the per-sample copy (plan._DEN_COPY), fp32 and bf16-backward plans."""
    import drsa_audio_amd.engine.plan as plan
    from drsa_audio_amd.engine import clear_cache
    from drsa_audio_amd.utils.constants import LRP_NAME_MAP_VGGISH
    from drsa_audio_amd.xai.explain.attribute import compute_relevances
    from drsa_audio_amd.zennit.canonizers import SequentialMergeBatchNorm
    from drsa_audio_amd.zennit.composites import NameMapComposite
    from lrp_common import logmel, vggish
    if bf16_bwd:
        monkeypatch.setenv("DRSA_AMD_BF16_BACKWARD", "1")
    net = vggish()
    if bf16_bwd:
        net = net.bfloat16()
    net = net.to(DEV)
    x = logmel(2, 128, 256, seed=9).to(DEV)
    comp = NameMapComposite(LRP_NAME_MAP_VGGISH, canonizers=[SequentialMergeBatchNorm()])
    outs = []
    for copy_den in (False, True):
        monkeypatch.setattr(plan, "_DEN_COPY", copy_den)
        clear_cache()
        outs.append(compute_relevances(net, x, comp, class_idx=2).cpu())
    clear_cache()
    assert torch.equal(outs[0], outs[1])
