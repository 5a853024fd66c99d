"""PixelFlipping end to end on the GPU (reference pf.py:29-292 + core.py): per LRP configuration
(SpecialFirstLayerMapComposite, or NameLayerMapComposite with a 'name_map' key; rules from
rule_mapper incl. Norm and ZPlus, Pass on the activations) the heatmaps of every class block are
bit-identical to the exact oracle (Pass vs the ReLU mask differ at most in the sign of a zero),
and the AUPC equals oracle/flip_ref.py's restatement of the reference Flipper run with the same
forward function.  Concept flipping: HeatmapGenerator subspace heatmaps -> Flipper."""
import copy

import numpy as np
import pytest
import torch

import flip_ref
import lrp_ref
from lrp_common import gtzan128, logmel, ortho, u64
from drsa_audio_amd.utils.constants import LRP_NAME_MAP_GTZAN
from drsa_audio_amd.xai.pixelflipping import PixelFlipping, concept_flipping
from drsa_audio_amd.zennit.rules import Gamma

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _spec_rule(r):
    k = r.kind
    if k == "epsilon":
        return ("epsilon", r.epsilon)
    if k == "norm":
        return ("epsilon", r.stabilizer)
    if k == "gamma":
        return ("gamma", r.gamma, r.stabilizer)
    if k in ("wsquare", "flat", "zplus"):
        return (k, r.stabilizer)
    if k == "pass":
        return ("pass",)
    if k == "alphabeta":
        return ("alphabeta", r.alpha, r.beta, r.stabilizer)
    raise ValueError(k)


def _check_order(order_dev, R, ps):
    """The device ranking (float32 patch sums) equals the float64 one except at near-ties."""
    o_ref = flip_ref.patch_order(R, ps)
    o = order_dev.cpu()
    if torch.equal(o, o_ref):
        return
    sums = flip_ref.patch_sums(R, ps)
    s_dev = torch.gather(sums, -1, o)
    s_ref = torch.gather(sums, -1, o_ref)
    assert torch.allclose(s_dev, s_ref, rtol=1e-5, atol=1e-9 * float(sums.abs().max()))


CONFIGS = [
    {"convolutional": ("gamma", 0.25), "dense": ("epsilon", 1e-7), "first_layer": ("wsquare",)},
    {"convolutional": ("zplus",), "dense": ("norm",), "first_layer": ("flat",)},
    {"convolutional": ("alphabeta", 2.0), "dense": ("epsilon", 1e-7), "first_layer": ("wsquare",)},
    {"convolutional": ("epsilon", 1e-6), "dense": ("epsilon", 1e-7), "first_layer": ("wsquare",),
     "name_map": [(["features.3"], Gamma(gamma=0.5, stabilizer=1e-7))]},
]


@pytest.mark.parametrize("ci", range(len(CONFIGS)))
def test_pixelflipping_config_vs_oracle(ci):
    conf = CONFIGS[ci]
    net = gtzan128()
    x = logmel(10, seed=60 + ci)
    pf = PixelFlipping(net, x, perturbation_size=16, num_classes=10, device=DEV)
    aupc, preds, flips, heatmaps = pf([conf], plot=False)
    name = pf._get_configuration_name(conf)
    R = heatmaps[name].cpu()
    rules = {n: _spec_rule(r) for n, r in pf._get_composite(conf).rules(net).items()}
    net_cpu = copy.deepcopy(net).cpu()
    for i in range(10):
        _, Rref = lrp_ref.lrp(net_cpu, rules, x[i:i + 1], class_idx=i, mode="exact")
        assert torch.equal(R[i:i + 1], Rref), (name, i)
    order = pf.pixel_flipper.sorted_patch_indices_by_relevance
    _check_order(order, R, 16)
    a_ref, m_ref, f_ref, _ = flip_ref.flip(pf._forward_func(pf.canonizer), x.to(DEV), R, 16, order=order.cpu())
    assert np.array_equal(flips, f_ref)
    assert np.array_equal(aupc[name], a_ref) and np.array_equal(preds[name], m_ref)
    assert aupc[name].shape == (10, 1) and np.all(np.isfinite(aupc[name]))


def test_engine_forward_aupc_close_to_torch_forward():
    """forward='engine' (HIP forward, steps fused in chunks of fuse_max_rows rows) against the
    default model(x) forward: AUPC within 1e-4 relative + 1e-4 absolute (fp32 accumulation order)."""
    net = gtzan128()
    x = logmel(10, seed=71)
    conf = CONFIGS[0]
    out = {}
    for fw in ("torch", "engine"):
        pf = PixelFlipping(net, x, perturbation_size=16, num_classes=10, device=DEV, forward=fw, fuse_max_rows=50)
        aupc, preds, flips, _ = pf([conf], plot=False)
        out[fw] = (aupc[pf._get_configuration_name(conf)], preds[pf._get_configuration_name(conf)])
    np.testing.assert_allclose(out["engine"][0], out["torch"][0], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(out["engine"][1], out["torch"][1], rtol=1e-4, atol=1e-4)


def test_engine_forward_equals_torch_forward_scores():
    net = gtzan128()
    x = logmel(10, seed=70)
    pf = PixelFlipping(net, x, perturbation_size=16, num_classes=10, device=DEV, forward="engine")
    fe = pf._forward_func(None)
    pf.forward = "torch"
    ft = pf._forward_func(None)
    with torch.no_grad():
        np.testing.assert_allclose(fe(x.to(DEV)).cpu(), ft(x.to(DEV)).cpu(), rtol=1e-4, atol=1e-4)


def test_concept_flipping_runs_on_subspace_heatmaps():
    net = gtzan128().to(DEV)
    x = logmel(10, seed=80)
    from drsa_audio_amd.utils.constants import CLASS_IDX_MAPPER
    Us = {g: (u64() if k % 2 == 0 else ortho(64, k)) for g, k in CLASS_IDX_MAPPER.items()}
    aupc, preds, flips = concept_flipping(net, x, LRP_NAME_MAP_GTZAN, 7, Us=Us, num_concepts=4, device=DEV)
    assert aupc.shape == (10, 1) and np.all(np.isfinite(aupc)) and flips.sum() == 64
    assert preds.shape == (len(flips),)


def test_compute_relevances_results_do_not_alias():
    """Consecutive calls with the same shape must return independent tensors (the engine reuses
    its buffers internally)."""
    from drsa_audio_amd.xai.explain.attribute import compute_relevances
    from drsa_audio_amd.zennit.composites import NameMapComposite
    net = gtzan128().to(DEV)
    comp = NameMapComposite(LRP_NAME_MAP_GTZAN)
    x = logmel(2, seed=90).to(DEV)
    r0 = compute_relevances(net, x, comp, class_idx=0)
    keep = r0.clone()
    r1 = compute_relevances(net, x, comp, class_idx=5)
    assert r0.data_ptr() != r1.data_ptr() and torch.equal(r0, keep) and not torch.equal(r0, r1)
