"""The WSquare first layer's w^2 contraction fused into the second layer's backward epilogue
(drsa_amd_conv_bwd_first_fused: the tile's R re-laid as the first layer's unpooled g in LDS,
contracted there; R stored only on the tiles' border cell rings, from which a second kernel
computes the footprints' border pixels).

Parity: the input relevance is bit-identical to drsa_amd_conv_bwd (POST_DIV on the full copy) /
drsa_amd_conv_bwd_den_ring followed by drsa_amd_first_layer_bwd (the dense chain the oracle's
lrp_exact.c restates, pinned in test_lrp_gpu / test_pins_gpu), for the ring and the full-copy
denominator, one and two clones per sample, several image sizes; the output starts as NaN so an
unwritten pixel shows.  At plan level the engine (GTZAN standard LRP and HeatmapGenerator) gives
identical relevances with the fusion on and off (DRSA_AMD_FIRST_FUSE)."""
import numpy as np
import pytest
import torch

from drsa_audio_amd import _capi

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _first_layer(S, C, H2, W2, seed):
    """Input, the first layer's fp32 forward (map den, 2x2 pool) in both den forms, and w^2."""
    g = torch.Generator().manual_seed(seed)
    H, W = 2 * H2, 2 * W2
    x = (torch.randn(S, 1, H, W, generator=g) * 2).to(DEV)
    w = torch.randn(C, 1, 3, 3, generator=g)
    b = torch.randn(C, generator=g) * 0.1
    wts = torch.zeros(1, 9, 32)
    wts[0, :, :C] = w.reshape(C, 9).T
    b3 = torch.zeros(3, 32)
    b3[0, :C] = b
    wts, b3 = wts.to(DEV).contiguous(), b3.to(DEV).contiguous()
    w2 = (w ** 2).reshape(C, 9).to(DEV).contiguous()
    bb2 = (b ** 2).to(DEV).contiguous()
    dmap = torch.empty(C, H, W, device=DEV)
    s = _capi.stream_ptr(DEV)
    _capi.call("drsa_amd_first_layer_den", w2.data_ptr(), bb2.data_ptr(), dmap.data_ptr(), C, 1, H, W, s)
    y = torch.empty(S, C, H2, W2, device=DEV)
    am = torch.empty(S, C, H2, W2, dtype=torch.uint8, device=DEV)
    den = torch.empty(S, C, H2, W2, device=DEV)
    _capi.call("drsa_amd_conv_fwd", x.data_ptr(), wts.data_ptr(), b3.data_ptr(), dmap.data_ptr(), y.data_ptr(),
               am.data_ptr(), den.data_ptr(), S, 1, C, H, W, 1, 1, s)
    y2 = torch.empty_like(y)
    am2 = torch.empty_like(am)
    ring = torch.full((S, C, 2 * W2 + 8 * (H2 - 2)), float("nan"), device=DEV)
    _capi.call("drsa_amd_conv_fwd_den_ring", x.data_ptr(), wts.data_ptr(), b3.data_ptr(), dmap.data_ptr(),
               y2.data_ptr(), am2.data_ptr(), ring.data_ptr(), S, C, H, W, 1, s)
    torch.cuda.synchronize()
    assert torch.equal(y, y2) and torch.equal(am, am2)
    c4 = dmap[:, 1, 1].reshape(-1, 1).expand(-1, 4).contiguous()
    return y, am, den, ring, c4, w2


def _tile_ring(H2, W2):
    m = torch.zeros(H2, W2, dtype=torch.bool, device=DEV)
    rows = torch.arange(H2, device=DEV) % 8
    cols = torch.arange(W2, device=DEV) % 32
    m[(rows == 0) | (rows == 7), :] = True
    m[:, (cols < 4) | (cols >= 28)] = True
    return m


@pytest.mark.parametrize("cin,H2,W2", [(32, 64, 64), (64, 32, 32), (32, 16, 32), (32, 8, 64), (64, 24, 96)])
@pytest.mark.parametrize("ring", [True, False])
@pytest.mark.parametrize("clones", [1, 2])
def test_fused_first_layer_equals_conv_bwd_plus_first_layer(cin, H2, W2, ring, clones):
    lib = _capi.lib()
    C, S = 32, 3
    assert lib.drsa_amd_conv_bwd_has_kernel_first_fused(cin, C, H2, W2) == 1
    Bq = S * clones
    y, am, den, dring, c4, w2 = _first_layer(S, C, H2, W2, seed=cin + H2 + W2)
    g = torch.Generator().manual_seed(cin * 5 + W2 + clones)
    gin = torch.randn(Bq, cin, H2 // 2, W2 // 2, generator=g).to(DEV)
    gam = torch.randint(0, 4, (S, cin, H2 // 2, W2 // 2), generator=g, dtype=torch.uint8).to(DEV)
    wts = (torch.randn(lib.drsa_amd_conv_weight_floats(cin, C, 1), generator=g) * 0.1).to(DEV)
    s = _capi.stream_ptr(DEV)
    eps = 1e-7
    R_ref = torch.full((Bq, C, H2, W2), float("nan"), device=DEV)
    if ring:
        _capi.call("drsa_amd_conv_bwd_den_ring", gin.data_ptr(), gam.data_ptr(), wts.data_ptr(), 0, y.data_ptr(),
                   dring.data_ptr(), c4.data_ptr(), R_ref.data_ptr(), Bq, clones, cin, C, H2, W2, 1, _capi.XM_MUL,
                   eps, s)
    else:
        _capi.call("drsa_amd_conv_bwd", gin.data_ptr(), gam.data_ptr(), wts.data_ptr(), y.data_ptr(), den.data_ptr(),
                   R_ref.data_ptr(), Bq, clones, cin, C, H2, W2, 1, _capi.XM_MUL, _capi.POST_DIV, eps, s)
    first_ref = torch.full((Bq, 1, 2 * H2, 2 * W2), float("nan"), device=DEV)
    _capi.call("drsa_amd_first_layer_bwd", R_ref.data_ptr(), am.data_ptr(), w2.data_ptr(), first_ref.data_ptr(), Bq,
               clones, C, 2 * H2, 2 * W2, s)
    R_ring = torch.full_like(R_ref, float("nan"))
    first = torch.full_like(first_ref, float("nan"))
    _capi.call("drsa_amd_conv_bwd_first_fused", gin.data_ptr(), gam.data_ptr(), wts.data_ptr(), y.data_ptr(),
               (dring if ring else den).data_ptr(), c4.data_ptr() if ring else None, am.data_ptr(), w2.data_ptr(),
               R_ring.data_ptr(), first.data_ptr(), Bq, clones, cin, C, H2, W2, eps, s)
    torch.cuda.synchronize()
    assert not torch.isnan(first_ref).any()
    assert (first_ref != 0).float().mean() > 0.3          # a real test: most pixels carry relevance
    assert not torch.isnan(first).any()
    assert torch.equal(first, first_ref)
    m = _tile_ring(H2, W2)
    assert torch.equal(R_ring[..., m], R_ref[..., m])


def test_fused_first_layer_rejects():
    lib = _capi.lib()
    assert lib.drsa_amd_conv_bwd_has_kernel_first_fused(32, 32, 64, 48) == 0     # W % 32
    assert lib.drsa_amd_conv_bwd_has_kernel_first_fused(32, 64, 64, 64) == 0     # cout != 32
    assert lib.drsa_amd_conv_bwd_has_kernel_first_fused(128, 32, 64, 64) == 0    # no instance
    assert lib.drsa_amd_conv_bwd_has_kernel_first_fused(32, 32, 64, 128) == 0    # border workgroup width
    assert lib.drsa_amd_conv_bwd_first_fused(None, None, None, None, None, None, None, None, None, None, 2, 1, 32, 32,
                                             8, 32, 0.0, None) == -1


@pytest.mark.parametrize("hg", [False, True])
def test_plan_first_fused_equals_unfused(monkeypatch, hg):
    import copy
    import drsa_audio_amd.engine.plan as plan
    from drsa_audio_amd.engine import clear_cache
    from drsa_audio_amd.utils.constants import LRP_NAME_MAP_GTZAN
    from drsa_audio_amd.xai.explain.attribute import compute_relevances
    from drsa_audio_amd.xai.explain.explainer import HeatmapGenerator
    from drsa_audio_amd.zennit.composites import NameMapComposite
    from lrp_common import gtzan128, logmel, u64
    net = gtzan128().to(DEV)
    x = logmel(6, seed=23).to(DEV)
    outs = []
    for fuse in (True, False):
        monkeypatch.setattr(plan, "_FIRST_FUSE", fuse)
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
