"""Custom-Hook slow path (engine/hooks.py), host-side parts: which rules route there, and the
built-in rule arithmetic it applies per module, against the oracle's zennit-structured
restatement (oracle/lrp_ref.py rule_backward_zennit) on small conv and dense layers."""
import pytest
import torch
import torch.nn as nn

import lrp_ref
from drsa_audio_amd.engine.hooks import has_custom_hooks, is_custom_hook, rule_relevance
from drsa_audio_amd.xai.explain.attribute import SubspaceHook
from drsa_audio_amd.zennit.core import Hook
from drsa_audio_amd.zennit.rules import AlphaBeta, Epsilon, Flat, Gamma, Norm, Pass, WSquare, ZPlus


class Doubling(Hook):
    def backward(self, module, grad_input, grad_output):
        return tuple(2 * g for g in grad_input)


class MySubspace(SubspaceHook):
    def backward(self, module, grad_input, grad_output):
        return grad_output


def test_routing():
    for r in (Epsilon(), Gamma(), WSquare(), Flat(), ZPlus(), AlphaBeta(), Norm(), Pass(), SubspaceHook(4), None,
              Hook()):
        assert not is_custom_hook(r), r
    assert is_custom_hook(Doubling())
    assert is_custom_hook(MySubspace(4))
    assert has_custom_hooks({"a": Epsilon(), "b": Doubling()})
    assert not has_custom_hooks({"a": Epsilon(), "b": SubspaceHook(4)})


def _layer(kind):
    torch.manual_seed(3)
    if kind == "conv":
        m = nn.Conv2d(4, 6, 3, padding=1)
        x = torch.randn(2, 4, 7, 9)
        L = lrp_ref.Layer("c", m, "conv")
    else:
        m = nn.Linear(12, 5)
        x = torch.randn(3, 12)
        L = lrp_ref.Layer("l", m, "linear")
    return m, x, L


RULES = [
    (Epsilon(1e-3), ("epsilon", 1e-3)),
    (Norm(1e-4), ("epsilon", 1e-4)),
    (Gamma(0.25, 1e-6), ("gamma", 0.25, 1e-6)),
    (WSquare(1e-6), ("wsquare", 1e-6)),
    (Flat(1e-6), ("flat", 1e-6)),
    (ZPlus(1e-6), ("zplus", 1e-6)),
    (AlphaBeta(2.0, 1.0, 1e-6), ("alphabeta", 2.0, 1.0, 1e-6)),
]


@pytest.mark.parametrize("kind", ["conv", "linear"])
@pytest.mark.parametrize("rule,spec", RULES, ids=[r[1][0] + str(i) for i, r in enumerate(RULES)])
def test_rule_relevance_matches_oracle(kind, rule, spec):
    m, x, L = _layer(kind)
    with torch.no_grad():
        z = m(x)
    R = torch.randn_like(z)
    got = rule_relevance(rule, m, x, R)
    want = lrp_ref.rule_backward_zennit(L, spec, x, z, R)
    assert got.shape == x.shape
    torch.testing.assert_close(got, want, rtol=1e-5, atol=1e-6)


def test_epsilon_on_projection_module():
    """Epsilon on a Projection (non-affine module): x (.) J^T(R / stab(z)), J from autograd."""
    from drsa_audio_amd.model.modify_model import Projection
    torch.manual_seed(0)
    U, _ = torch.linalg.qr(torch.randn(8, 8))
    p = Projection(U, 2)
    x = torch.randn(2, 8, 4, 4)
    with torch.no_grad():
        z = p(x)
    R = torch.randn_like(z)
    got = rule_relevance(Epsilon(1e-6), p, x, R)
    L = lrp_ref.Layer("features.projection", p, "proj")
    want = lrp_ref.rule_backward_analytic(L, ("epsilon", 1e-6), x, z, R)
    torch.testing.assert_close(got, want, rtol=1e-5, atol=1e-6)


def test_slow_path_refuses_host_model():
    from drsa_audio_amd import _capi
    from drsa_audio_amd.engine.hooks import HookedAutograd
    from drsa_audio_amd.zennit.composites import NameMapComposite
    m = nn.Sequential(nn.Linear(3, 2))
    with pytest.raises(_capi.DrsaAmdError):
        HookedAutograd(m, NameMapComposite([(["0"], Doubling())]))
