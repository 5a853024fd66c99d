"""Pixel/concept flipping (reference cxai/xai/pixelflipping) on the CPU: the product Flipper
against the loop-for-loop restatement oracle/flip_ref.py (reference core.py:6-312), the flip
schedule, composites (SpecialFirstLayerMapComposite / NameLayerMapComposite / zennit types) and
PixelFlipping's rule/configuration helpers (reference pf.py:196-292)."""
import numpy as np
import pytest
import torch
import torch.nn as nn

import flip_ref
from lrp_common import gtzan128
from drsa_audio_amd.xai.pixelflipping import Flipper, PixelFlipping
from drsa_audio_amd.zennit.composites import LayerMapComposite, NameLayerMapComposite, SpecialFirstLayerMapComposite
from drsa_audio_amd.zennit.rules import AlphaBeta, Epsilon, Flat, Gamma, Norm, Pass, WSquare
from drsa_audio_amd.zennit.types import Activation, Convolution, Linear


def _linear_model(n_classes, C, H, W, seed=0):
    g = torch.Generator().manual_seed(seed)
    Wm = torch.randn(C * H * W, n_classes, generator=g, dtype=torch.float64) / (C * H * W) ** 0.5
    b = torch.linspace(0.5, 1.5, n_classes, dtype=torch.float64)
    return lambda x: (x.reshape(x.size(0), -1).double() @ Wm + b).float()


def _distinct_relevance(B, n_c, H, W, seed):
    # integer-valued relevance: distinct patch sums, so the ranking has no ties to break
    g = torch.Generator().manual_seed(seed)
    return torch.randint(-50, 200, (B, n_c, H, W), generator=g).float()


@pytest.mark.parametrize("n_c,H,W,ps", [(1, 32, 48, 8), (4, 32, 32, 8), (3, 36, 40, 8), (1, 64, 64, 16)])
def test_flipper_matches_reference_restatement(n_c, H, W, ps):
    n_classes, spc, C = 2, 3, 1
    B = n_classes * spc
    x = torch.randn(B, C, H, W, generator=torch.Generator().manual_seed(1))
    R = _distinct_relevance(B, n_c, H, W, 2)
    f = _linear_model(n_classes, C, H, W)
    fl = Flipper(perturbation_size=ps, device="cpu")
    aupc, mean_pred, flips = fl(f, x, R)
    a_ref, m_ref, f_ref, _ = flip_ref.flip(f, x, R, ps)
    assert np.array_equal(flips, f_ref)
    assert torch.equal(fl.sorted_patch_indices_by_relevance, flip_ref.patch_order(R, ps))
    assert aupc.shape == (n_classes, spc) and np.array_equal(aupc, a_ref)
    assert np.array_equal(mean_pred, m_ref)
    # all steps in one forward call: the same numbers for a per-sample forward
    aupc2, mean2, _ = Flipper(perturbation_size=ps, device="cpu", fuse_steps=True)(f, x, R)
    np.testing.assert_allclose(aupc2, aupc, rtol=1e-6, atol=1e-7)


def test_flip_schedule():
    assert Flipper.schedule(64) == [0, 1, 4, 9, 16, 25, 9]
    assert Flipper.schedule(1) == [0, 1]
    assert Flipper.schedule(5) == [0, 1, 4]
    assert sum(Flipper.schedule(1000)) == 1000


def test_random_mode_and_inpainting_refused():
    x = torch.randn(4, 1, 16, 16)
    f = _linear_model(2, 1, 16, 16)
    aupc, _, flips = Flipper(perturbation_size=4, device="cpu")(f, x, None, flipping_mode="random")
    assert aupc.shape == (2, 2) and flips.sum() == 16
    with pytest.raises(NotImplementedError):
        Flipper(perturbation_mode="inpainting", device="cpu")(f, x, torch.rand(4, 1, 16, 16))
    with pytest.raises(ValueError):
        Flipper(perturbation_mode="blur")


def test_zennit_types_and_composites():
    net = gtzan128()
    assert isinstance(nn.Conv2d(1, 1, 3), Linear) and isinstance(nn.Conv2d(1, 1, 3), Convolution)
    assert not isinstance(nn.Linear(2, 2), Convolution) and isinstance(nn.ReLU(), Activation)
    first, conv, dense, pas = WSquare(), Gamma(gamma=0.25), Epsilon(epsilon=1e-7), Pass()
    lm = [(Activation, pas), (Convolution, conv), (Linear, dense)]
    r = SpecialFirstLayerMapComposite(layer_map=lm, first_map=[(Convolution, first)]).rules(net)
    convs = [n for n, m in net.named_modules() if isinstance(m, nn.Conv2d)]
    assert r[convs[0]] is first and all(r[n] is conv for n in convs[1:])
    assert all(r[n] is dense for n, m in net.named_modules() if isinstance(m, nn.Linear))
    assert all(r[n] is pas for n, m in net.named_modules() if isinstance(m, nn.ReLU))
    assert not any(isinstance(m, nn.MaxPool2d) for n, m in net.named_modules() if n in r)
    flat = Flat()
    r2 = NameLayerMapComposite(name_map=[(["features.0", "classifier.6"], flat)], layer_map=lm).rules(net)
    assert r2["features.0"] is flat and r2["classifier.6"] is flat and r2["features.3"] is conv
    assert LayerMapComposite(lm).rules(net)["features.0"] is conv


def test_pixelflipping_rules_and_names():
    net = gtzan128()
    pf = PixelFlipping(net, torch.zeros(10, 1, 128, 128), num_classes=10, device="cpu")
    pf.stabilizers = None
    ab = pf._get_rule("convolutional", {"convolutional": ("alphabeta", 2.0)})
    assert isinstance(ab, AlphaBeta) and ab.alpha == 2.0 and ab.beta == 1.0
    nm = pf._get_rule("dense", {"dense": ("norm",)})
    assert isinstance(nm, Norm) and nm.stabilizer == 1e-7
    with pytest.raises(ValueError):
        pf._get_rule("dense", {"dense": ("lrp-zb", 1)})
    conf = {"convolutional": ("gamma", 0.25), "dense": ("epsilon", 1e-7), "first_layer": ("wsquare",)}
    assert pf._get_configuration_name(conf) == "gamma_0.25_epsilon_1e-07_wsquare"
    assert pf._get_configuration_name({"convolutional": ("alphabeta", 2.0), "dense": ("zplus",),
                                       "first_layer": ("flat",)}) == "alpha_2.0_beta_1.0zplus_flat"
    pf.canonizer = None
    with pytest.raises(AssertionError):
        pf._get_composite({"convolutional": ("gamma", 0.25)})
