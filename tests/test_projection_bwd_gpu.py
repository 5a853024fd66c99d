"""drsa_amd_projection_bwd: the recompute path (h and a' rebuilt from a, the engine default) against
the stored-buffer path, bitwise, over d (16 / 64 / 128: the register and the L1 a / den paths),
K (d_k = 4, 8, 16, 32: the generic clone loop and its d_k = 16 form), fan-out modes, the pooled and
the dense relevance input, and with and without the lower layer's denominator (den = NULL divides by
nothing: x / 1 == x).  Reference: cxai/xai/explain/attribute.py:53-58 (SubspaceHook mask),
cxai/model/modify_model.py:75-123 (ProjectionModel)."""
import numpy as np
import pytest
import torch

from drsa_audio_amd import _capi

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _ortho(d, seed):
    q = np.linalg.qr(np.random.default_rng(seed).standard_normal((d, d)))[0]
    return torch.from_numpy(q.astype(np.float32)).to(DEV)


@pytest.mark.parametrize("D,K", [(16, 4), (64, 4), (64, 8), (64, 2), (128, 4)])
@pytest.mark.parametrize("pool", [0, 1])
@pytest.mark.parametrize("has_den", [True, False])
@pytest.mark.parametrize("fanout", [0, 1, 2])
def test_recompute_equals_stored(D, K, pool, has_den, fanout):
    B, H, W = 3 if fanout == 0 else 2, 16, 16
    g = torch.Generator().manual_seed(D + 7 * K + 3 * pool + fanout)
    a = torch.randn(B, D, H, W, generator=g)
    # post-ReLU activations; the float64 check (fan-out 2) keeps a' away from 0, where fp32 and f64
    # stabilised quotients R / stab(a') legitimately part
    a = (a.abs() + 0.05 if fanout == 2 else a.clamp_min(0)).to(DEV)
    U = _ortho(D, D + K)
    s = _capi.stream_ptr(DEV)
    P = torch.empty_like(U)
    _capi.call("drsa_amd_projection_residual", U.data_ptr(), D, P.data_ptr(), s)
    h = torch.empty(B, D, H, W, device=DEV)
    ap = torch.empty(B, D, H, W, device=DEV)
    pooled = torch.empty(B, D, H // 2, W // 2, device=DEV) if pool else None
    amax = torch.empty(B, D, H // 2, W // 2, dtype=torch.uint8, device=DEV) if pool else None
    _capi.call("drsa_amd_projection_fwd", a.data_ptr(), U.data_ptr(), P.data_ptr(), h.data_ptr(), ap.data_ptr(),
               _capi.ptr(pooled), _capi.ptr(amax), B, D, H, W, pool, s)
    gshape = (B, D, H // 2, W // 2) if pool else (B, D, H, W)
    gp = torch.randn(*gshape, generator=g).to(DEV)
    den = (torch.randn(B, D, H, W, generator=g) * 2).to(DEV) if has_den else None
    nq = K + 1 if fanout == 1 else K if fanout == 2 else 1
    outs = []
    for stored in (True, False):
        G = torch.full((B * (nq if fanout else 1), D, H, W), float("nan"), device=DEV)
        _capi.call("drsa_amd_projection_bwd", gp.data_ptr(), _capi.ptr(amax), ap.data_ptr() if stored else None,
                   h.data_ptr() if stored else None, a.data_ptr(), _capi.ptr(den), U.data_ptr(), P.data_ptr(),
                   G.data_ptr(), B, D, H, W, K, 1e-6, 1e-7, fanout, s)
        outs.append(G)
    torch.cuda.synchronize()
    assert not torch.isnan(outs[1]).any()
    assert torch.equal(outs[0], outs[1])
    # semantics of one concept clone in float64: G_q = [a > 0] a (U_q U_q^T g2) / stab(den)
    if fanout == 2:
        a64, U64 = a.double(), U.double()
        R = gp.double()
        if pool:
            up = torch.zeros(B, D, H, W, dtype=torch.float64, device=DEV)
            am = amax.long()
            for sb in range(4):
                m = (am == sb).double() * R
                up[:, :, sb // 2::2, sb % 2::2] = m
            R = up
        ap64 = torch.einsum("ck,bkhw->bchw", U64 @ U64.T, a64)
        h64 = torch.einsum("cj,bchw->bjhw", U64, a64)
        stab = lambda t, e: t + torch.where(t >= 0, e, -e)
        g1 = R / stab(ap64, 1e-6)
        t = torch.einsum("cj,bchw->bjhw", U64, g1)
        g2 = h64 * t / stab(h64, 1e-6)
        dk = D // K
        q = 1
        Uq = U64[:, q * dk:(q + 1) * dk]
        c = torch.einsum("cj,bjhw->bchw", Uq, g2[:, q * dk:(q + 1) * dk])
        ref = a64 * c
        if has_den:
            ref = ref / stab(den.double(), 1e-7)
        ref = torch.where(a64 > 0, ref, torch.zeros_like(ref))
        got = outs[1].view(B, K, D, H, W)[:, q].double()
        scale = ref.abs().max().item() + 1e-30
        assert (got - ref).abs().max().item() / scale < 1e-4
