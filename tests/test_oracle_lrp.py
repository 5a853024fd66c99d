"""The LRP oracle (oracle/lrp_ref.py) on CPU.

zennit is not installed and the reference has no tests, so the rule arithmetic is
*parity-unpinned vs zennit*; it is pinned here by theory known-answer tests:
(i) sum of subspace heatmaps = standard heatmap, (ii) epsilon conservation, (iii) WSquare /
Flat input independence, (iv) U = I, K = 1 reproduces plain LRP, (v) a hand-computed
network in float64, plus agreement of the three oracle modes.
"""
import numpy as np
import pytest
import torch
import torch.nn as nn

import lrp_ref
from lrp_common import f64_anchored_check, gtzan128, logmel, maxnorm_err, ortho, spec, toy, u64
from drsa_audio_amd.model.modify_model import ProjectionModel
from drsa_audio_amd.utils.constants import LRP_NAME_MAP_GTZAN, LRP_NAME_MAP_TOY

NM = spec(LRP_NAME_MAP_GTZAN)


@pytest.fixture(scope="module")
def model():
    return gtzan128()


def test_zennit_structured_mode_equals_analytic(model):
    x = logmel(2)
    _, Ra = lrp_ref.lrp(model, NM, x, class_idx=3, mode="analytic")
    _, Rz = lrp_ref.lrp(model, NM, x, class_idx=3, mode="zennit")
    assert torch.equal(Ra, Rz)


def test_exact_mode_f64_anchored(model):
    """The pinned kernel order (mode exact == the HIP kernels bit for bit) is as accurate as the
    reference's own fp32 order, both measured against float64 (lrp_common.f64_anchored_check)."""
    x = logmel(8, seed=7)
    la, Ra = lrp_ref.lrp(model, NM, x, class_idx=5, mode="analytic")
    le, Re = lrp_ref.lrp(model, NM, x, class_idx=5, mode="exact")
    l64, R64 = lrp_ref.lrp(model, NM, x, class_idx=5, mode="f64")
    assert (la - le).abs().max() <= 1e-6 * la.abs().max()
    assert (la.double() - l64).abs().max() <= 1e-5 * l64.abs().max()
    f64_anchored_check(Re, Ra, R64)


@pytest.mark.parametrize("mode", ["analytic", "exact"])
def test_subspace_heatmaps_sum_to_standard(model, mode):
    pm = ProjectionModel(model, 7, u64(), 4).eval()
    out = lrp_ref.subspace_heatmaps(pm, NM, 4, logmel(1, seed=3), class_idx=2, mode=mode)
    s = out["subspace_heatmaps"].sum(1)
    std = out["standard_heatmaps"][:, 0]
    assert np.abs(s - std).max() <= 1e-5 * np.abs(std).max()
    assert np.allclose(out["subspace_relevances"].sum(1), out["standard_relevance"], rtol=1e-4, atol=1e-9)


def test_epsilon_conservation_bias_free_linear():
    torch.manual_seed(0)
    lin = nn.Linear(7, 5, bias=False)
    L = lrp_ref.Layer("l", lin, "linear")
    x = torch.randn(3, 7)
    z = lin(x).detach()
    R = torch.randn(3, 5)
    eps = 1e-3
    Rin = lrp_ref.rule_backward_analytic(L, ("epsilon", eps), x, z, R)
    expect = (R * z / lrp_ref.stabilize(z, eps)).sum(1)
    assert torch.allclose(Rin.sum(1), expect, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("kind", ["wsquare", "flat"])
def test_first_layer_rules_ignore_input_values(kind):
    torch.manual_seed(1)
    conv = nn.Conv2d(1, 4, 3, padding=1)
    L = lrp_ref.Layer("c", conv, "conv")
    R = torch.randn(2, 4, 8, 8)
    x1, x2 = torch.randn(2, 1, 8, 8), torch.randn(2, 1, 8, 8) * 10
    r1 = lrp_ref.rule_backward_analytic(L, (kind, 1e-7), x1, None, R)
    r2 = lrp_ref.rule_backward_analytic(L, (kind, 1e-7), x2, None, R)
    assert torch.equal(r1, r2)


def test_identity_projection_reproduces_plain_lrp(model):
    x = logmel(1, seed=11)
    _, R = lrp_ref.lrp(model, NM, x, class_idx=1)
    pm = ProjectionModel(model, 7, torch.eye(64), 1).eval()
    out = lrp_ref.subspace_heatmaps(pm, NM, 1, x, class_idx=1)
    assert maxnorm_err(out["standard_heatmaps"], R.numpy()) < 1e-4
    assert np.allclose(out["subspace_heatmaps"], out["standard_heatmaps"])


def _hand_lrp(W1, b1, W2, b2, x, c, gam, eps):
    """float64 loops: conv3x3(1->2)+ReLU+maxpool2 -> Linear(8->3); Gamma on conv, Epsilon on linear."""
    H = x.shape[0]
    z = np.zeros((2, H, H)); zp = np.zeros((2, H, H))
    Wp = W1 + gam * np.maximum(W1, 0); bp = b1 + gam * np.maximum(b1, 0)
    xp = np.pad(x, 1)
    for o in range(2):
        for i in range(H):
            for j in range(H):
                patch = xp[i:i + 3, j:j + 3]
                z[o, i, j] = (patch * W1[o]).sum() + b1[o]
                zp[o, i, j] = (np.maximum(patch, 0) * Wp[o]).sum() + bp[o] + (np.minimum(patch, 0) * (W1[o] + gam * np.minimum(W1[o], 0))).sum()
    a = np.maximum(z, 0)
    P = np.zeros((2, H // 2, H // 2)); arg = {}
    for o in range(2):
        for i in range(H // 2):
            for j in range(H // 2):
                win = a[o, 2 * i:2 * i + 2, 2 * j:2 * j + 2]
                k = int(np.argmax(win.reshape(-1)))
                P[o, i, j] = win.reshape(-1)[k]; arg[(o, i, j)] = (2 * i + k // 2, 2 * j + k % 2)
    f = P.reshape(-1)
    y = W2 @ f + b2
    Rout = np.zeros_like(y); Rout[c] = y[c]
    st = lambda t: t + eps * (np.sign(t) + (t == 0))
    Rf = f * (W2.T @ (Rout / st(y)))
    Ra = np.zeros_like(a)
    for (o, i, j), (p, q) in arg.items():
        Ra[o, p, q] = Rf.reshape(P.shape)[o, i, j] * (a[o, p, q] > 0)
    g = Ra * (z > 0) / st(zp)
    Rin = np.zeros((H, H))
    gp = np.pad(g, ((0, 0), (1, 1), (1, 1)))
    for i in range(H):
        for j in range(H):
            acc_p = 0.0; acc_n = 0.0
            for o in range(2):
                for ky in range(3):
                    for kx in range(3):
                        gv = gp[o, i + 2 - ky, j + 2 - kx]
                        acc_p += gv * Wp[o, ky, kx]
                        acc_n += gv * (W1[o, ky, kx] + gam * min(W1[o, ky, kx], 0))
            Rin[i, j] = max(x[i, j], 0) * acc_p + min(x[i, j], 0) * acc_n
    return y, Rin


def test_hand_computed_network_float64():
    rng = np.random.default_rng(5)
    W1 = rng.standard_normal((2, 3, 3)); b1 = rng.standard_normal(2) * 0.1
    W2 = rng.standard_normal((3, 8)); b2 = rng.standard_normal(3) * 0.1
    x = rng.standard_normal((4, 4))
    y, Rin = _hand_lrp(W1, b1, W2, b2, x, 1, 0.25, 1e-6)

    class Net(nn.Module):
        def __init__(self):
            super().__init__()
            self.features = nn.Sequential(nn.Conv2d(1, 2, 3, padding=1), nn.ReLU(), nn.MaxPool2d(2))
            self.classifier = nn.Sequential(nn.Linear(8, 3))
    net = Net()
    with torch.no_grad():
        net.features[0].weight.copy_(torch.from_numpy(W1[:, None]))
        net.features[0].bias.copy_(torch.from_numpy(b1))
        net.classifier[0].weight.copy_(torch.from_numpy(W2))
        net.classifier[0].bias.copy_(torch.from_numpy(b2))
    rules = {"features.0": ("gamma", 0.25, 1e-6), "classifier.0": ("epsilon", 1e-6)}
    lg, R = lrp_ref.lrp(net, rules, torch.from_numpy(x[None, None]).float(), class_idx=1)
    assert np.allclose(lg.numpy()[0], y, rtol=1e-5, atol=1e-5)
    assert np.abs(R.numpy()[0, 0] - Rin).max() <= 1e-4 * np.abs(Rin).max()


def test_sort_ties_and_batch_one():
    sub = np.zeros((1, 3, 2, 2), dtype=np.float32)
    sub[0, 0] = 1.0; sub[0, 2] = 1.0; sub[0, 1] = 2.0
    s, r, m = lrp_ref.sort_subspaces(sub)
    assert m.tolist() == [[1, 2, 0]]            # descending, ties -> larger index first
    assert s.shape == (1, 3, 2, 2) and r.shape == (1, 3)


def test_toy_runs_through_oracle():
    x = logmel(1, 64, 64, seed=2)
    lg, R = lrp_ref.lrp(toy(), spec(LRP_NAME_MAP_TOY), x, class_idx=0)
    assert R.shape == x.shape and torch.isfinite(R).all()


def test_model_fixture_pins_vggtype(golden_dir):
    fx = np.load(f"{golden_dir}/model_fixture.npz")
    m = gtzan128()
    assert [n for n, _ in m.named_modules() if n.count(".") == 1] == list(fx["gtzan_names"])
    assert np.array_equal(np.array([float(p.double().sum()) for p in m.parameters()]), fx["gtzan_param_sums"])
    with torch.no_grad():
        assert np.array_equal(m(torch.from_numpy(fx["gtzan_x"])).numpy(), fx["gtzan_logits"])
        pm = ProjectionModel(m, 7, u64(), 4).eval()
        assert np.array_equal(pm(torch.from_numpy(fx["gtzan_x"])).numpy(), fx["proj_logits"])
        assert [n for n, _ in pm.named_modules() if n.count(".") == 1] == list(fx["proj_names"])
        h = pm.features[:9](torch.from_numpy(fx["gtzan_x"]))
        assert np.array_equal(h[:, :64].numpy(), fx["proj_h"])
    t = toy()
    assert np.array_equal(np.array([float(p.double().sum()) for p in t.parameters()]), fx["toy_param_sums"])


def test_preprocessing_helpers_match_reference_fixture(golden_dir):
    import drsa_ref
    fx = np.load(f"{golden_dir}/preprocessing_fixture.npz")
    va = drsa_ref.get_vectors_from_maps(torch.from_numpy(fx["maps_a"]), fx["idx"])
    vr = drsa_ref.get_vectors_from_maps(torch.from_numpy(fx["maps_r"]), fx["idx"])
    assert np.array_equal(va.numpy(), fx["vec_a"]) and np.array_equal(vr.numpy(), fx["vec_r"])
    ctx = drsa_ref.compute_context_vectors(va, vr)
    assert np.array_equal(ctx.numpy(), fx["ctx"])
    assert np.array_equal(drsa_ref.normalize_vectors(va).numpy(), fx["norm_a"])


def test_merge_batch_norm_preserves_forward():
    """oracle.merge_batch_norm (zennit SequentialMergeBatchNorm restated): the merged network
    computes the same function as the BN network in eval mode."""
    from lrp_common import vggish
    net = vggish(input_size=(64, 128))
    merged = lrp_ref.merge_batch_norm(net)
    x = logmel(2, 64, 128, seed=1)
    with torch.no_grad():
        a = net.classifier(net.features(x).reshape(2, -1))
        b = merged.classifier(merged.features(x).reshape(2, -1))
    assert torch.allclose(a, b, rtol=1e-4, atol=1e-6)
    assert not any(isinstance(m, (torch.nn.BatchNorm1d, torch.nn.BatchNorm2d)) for m in merged.modules())


def test_product_bn_fold_matches_oracle_merge():
    from lrp_common import vggish
    from drsa_audio_amd.zennit.canonizers import SequentialMergeBatchNorm
    net = vggish(input_size=(64, 128))
    merged = lrp_ref.merge_batch_norm(net)
    w, b = SequentialMergeBatchNorm.fold(net.features[3].weight.detach(), net.features[3].bias.detach(),
                                         net.features[4])
    assert torch.equal(w, merged.features[3].weight) and torch.equal(b, merged.features[3].bias)


def _conv_layer(cin=3, cout=4, bias=False, seed=0):
    torch.manual_seed(seed)
    conv = nn.Conv2d(cin, cout, 3, padding=1, bias=bias)
    return conv, lrp_ref.Layer("c", conv, "conv")


def test_zplus_conservation_bias_free_conv():
    """ZPlus (zennit 0.5.1 semantics, restated): sum R_in = sum R * den / stab(den) with
    den = conv(x+; W+) + conv(x-; W-) when the conv has no bias."""
    conv, L = _conv_layer()
    x = torch.randn(2, 3, 6, 5, dtype=torch.float64)
    conv = conv.double()
    L = lrp_ref.Layer("c", conv, "conv")
    z = conv(x).detach()
    R = torch.randn_like(z)
    eps = 1e-6
    Rin = lrp_ref.rule_backward_analytic(L, ("zplus", eps), x, z, R)
    w = conv.weight.detach()
    den = nn.functional.conv2d(x.clamp(min=0), w.clamp(min=0), padding=1) + \
        nn.functional.conv2d(x.clamp(max=0), w.clamp(max=0), padding=1)
    expect = (R * den / lrp_ref.stabilize(den, eps)).sum((1, 2, 3))
    assert torch.allclose(Rin.sum((1, 2, 3)), expect, rtol=1e-10, atol=1e-12)


def test_zplus_zennit_structured_equals_analytic():
    conv, L = _conv_layer(bias=True, seed=3)
    x = torch.randn(2, 3, 8, 8)
    z = conv(x).detach()
    R = torch.randn_like(z)
    Ra = lrp_ref.rule_backward_analytic(L, ("zplus", 1e-6), x, z, R)
    Rz = lrp_ref.rule_backward_zennit(L, ("zplus", 1e-6), x, z, R)
    assert torch.allclose(Ra, Rz, rtol=1e-5, atol=1e-6)


def test_alphabeta_one_zero_is_zplus():
    """Known answer (zennit 0.5.1 semantics, restated): AlphaBeta(alpha=1, beta=0) is ZPlus."""
    conv, L = _conv_layer(bias=True, seed=7)
    x = torch.randn(2, 3, 8, 8)
    z = conv(x).detach()
    R = torch.randn_like(z)
    Rab = lrp_ref.rule_backward_analytic(L, ("alphabeta", 1.0, 0.0, 1e-6), x, z, R)
    Rzp = lrp_ref.rule_backward_analytic(L, ("zplus", 1e-6), x, z, R)
    assert torch.equal(Rab, Rzp)


def test_alphabeta_conservation_bias_free_conv():
    """sum R_in = sum R * (alpha * den+/stab(den+) - beta * den-/stab(den-)) without bias."""
    conv, L = _conv_layer(seed=9)
    conv = conv.double()
    L = lrp_ref.Layer("c", conv, "conv")
    x = torch.randn(2, 3, 6, 5, dtype=torch.float64)
    z = conv(x).detach()
    R = torch.randn_like(z)
    eps, alpha, beta = 1e-6, 2.0, 1.0
    Rin = lrp_ref.rule_backward_analytic(L, ("alphabeta", alpha, beta, eps), x, z, R)
    w = conv.weight.detach()
    c2 = nn.functional.conv2d
    dp = c2(x.clamp(min=0), w.clamp(min=0), padding=1) + c2(x.clamp(max=0), w.clamp(max=0), padding=1)
    dn = c2(x.clamp(min=0), w.clamp(max=0), padding=1) + c2(x.clamp(max=0), w.clamp(min=0), padding=1)
    expect = (R * (alpha * dp / lrp_ref.stabilize(dp, eps) - beta * dn / lrp_ref.stabilize(dn, eps))).sum((1, 2, 3))
    assert torch.allclose(Rin.sum((1, 2, 3)), expect, rtol=1e-10, atol=1e-12)


def test_alphabeta_zennit_structured_equals_analytic():
    conv, L = _conv_layer(bias=True, seed=11)
    x = torch.randn(2, 3, 8, 8)
    z = conv(x).detach()
    R = torch.randn_like(z)
    rule = ("alphabeta", 2.0, 1.0, 1e-6)
    Ra = lrp_ref.rule_backward_analytic(L, rule, x, z, R)
    Rz = lrp_ref.rule_backward_zennit(L, rule, x, z, R)
    assert torch.allclose(Ra, Rz, rtol=1e-5, atol=1e-5)


def test_zplus_is_the_large_gamma_limit_on_nonnegative_input():
    """Known answer: on x >= 0 with no bias, Gamma(gamma) -> ZPlus as gamma -> inf."""
    conv, L = _conv_layer(seed=5)
    conv = conv.double()
    L = lrp_ref.Layer("c", conv, "conv")
    x = torch.rand(2, 3, 7, 7, dtype=torch.float64)
    z = conv(x).detach()
    R = torch.rand_like(z) * (z > 0)
    Rzp = lrp_ref.rule_backward_analytic(L, ("zplus", 1e-12), x, z, R)
    Rg = lrp_ref.rule_backward_analytic(L, ("gamma", 1e7, 1e-12), x, z, R)
    assert (Rzp - Rg).abs().max() <= 1e-5 * Rzp.abs().max()


def _gamma_conv_1px(b):
    """Conv2d(1->1, 3x3, padding 1) on a 1x1 input: only the centre tap w_c = 1.5 meets the input."""
    conv = nn.Conv2d(1, 1, 3, padding=1).double()
    with torch.no_grad():
        conv.weight.copy_(torch.tensor([[[[0.3, -0.7, 0.2], [0.9, 1.5, -0.4], [0.1, 0.6, -0.2]]]]))
        conv.bias.fill_(b)
    return conv, lrp_ref.Layer("c", conv, "conv")


@pytest.mark.parametrize("mode", ["analytic", "zennit"])
def test_gamma_bias_known_answer(mode):
    """Known answer separating the two candidate Gamma bias conventions.

    zennit 0.5.1 ``rules.Gamma`` builds its five modified forwards from ``GammaMod(γ, min=0)``,
    ``GammaMod(γ, max=0, zero_params=zero_bias(...))``, ``GammaMod(γ, max=0)``,
    ``GammaMod(γ, min=0, zero_params=zero_bias(...))`` and the plain layer, i.e. the x⁻ terms
    carry no bias (the same ``zero_bias`` form as its ZPlus / AlphaBeta).  On x = 2 ≥ 0,
    w_c = 1.5, b = -0.5, γ = 0.25, R = 1:
      W⁺_c = 1.5 + 0.25·1.5 = 1.875,  b⁺ = -0.5,  b⁻ = -0.5 + 0.25·(-0.5) = -0.625
      z = 2·1.5 - 0.5 = 2.5 > 0
      zennit:            den₊ = 2·1.875 + b⁺          = 3.25   → R_in = 3.75 / 3.25  = 15/13
      bias in both terms: den₊ = 2·1.875 + b⁺ + b⁻    = 2.625  → R_in = 3.75 / 2.625 = 10/7
    """
    conv, L = _gamma_conv_1px(-0.5)
    x = torch.full((1, 1, 1, 1), 2.0, dtype=torch.float64)
    z = conv(x).detach()
    assert float(z) == 2.5
    fn = lrp_ref.rule_backward_analytic if mode == "analytic" else lrp_ref.rule_backward_zennit
    Rin = fn(L, ("gamma", 0.25, 1e-12), x, z, torch.ones_like(z))
    assert abs(float(Rin) - 15 / 13) < 1e-10
    assert abs(float(Rin) - 10 / 7) > 0.2


def test_gamma_bias_known_answer_slow_path_and_plan_bias():
    """The same known answer through the custom-Hook slow path's per-module arithmetic, and the
    plan's Gamma bias rows (engine/plan.py): row 1 = b⁺, row 2 (the x⁻ term's bias) = 0."""
    from drsa_audio_amd.engine.hooks import rule_relevance
    from drsa_audio_amd.zennit.rules import Gamma
    conv, _ = _gamma_conv_1px(-0.5)
    x = torch.full((1, 1, 1, 1), 2.0, dtype=torch.float64)
    Rin = rule_relevance(Gamma(0.25, 1e-12), conv, x, torch.ones(1, 1, 1, 1, dtype=torch.float64))
    assert abs(float(Rin) - 15 / 13) < 1e-10
    # a signed input exercises the x⁻ terms: den₊ = (x⁺·W⁺ + b⁺) + x⁻·W⁻ (no bias)
    torch.manual_seed(4)
    m = nn.Conv2d(2, 3, 3, padding=1).double()
    with torch.no_grad():
        m.bias.copy_(torch.tensor([-0.3, 0.2, -0.1]))
    xs = torch.randn(1, 2, 5, 5, dtype=torch.float64)
    zs = m(xs).detach()
    R = torch.rand_like(zs) * (zs > 0)
    L = lrp_ref.Layer("c", m, "conv")
    want = lrp_ref.rule_backward_analytic(L, ("gamma", 0.3, 1e-9), xs, zs, R)
    got = rule_relevance(Gamma(0.3, 1e-9), m, xs, R)
    torch.testing.assert_close(got, want, rtol=1e-10, atol=1e-12)
    w, b, g = m.weight.detach(), m.bias.detach(), 0.3
    c2 = nn.functional.conv2d
    bp = (b + g * b.clamp(min=0)).view(1, -1, 1, 1)
    den = (c2(xs.clamp(min=0), w + g * w.clamp(min=0), padding=1) + bp
           + c2(xs.clamp(max=0), w + g * w.clamp(max=0), padding=1))
    expect = (R * (den - bp) / lrp_ref.stabilize(den, 1e-9)).sum()   # conservation: the bias absorbs b⁺ once
    assert abs(float(want.sum() - expect)) <= 1e-9 * float(R.abs().sum())
