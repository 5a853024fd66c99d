"""Custom-Hook slow path (engine/hooks.py) on the GPU.

A composite that maps a module to a user-written Hook (its own ``backward``) cannot be compiled
into the HIP plan; ``get_engine`` routes it to ``HookedAutograd`` (torch autograd on the device
with zennit-style module hooks).  Gates:
* routing: the custom composite gets the slow path, the same name map without it the HIP plan;
* the slow path's built-in rules (no custom hook, forced) agree with the HIP plan, which is
  bit-exact vs the oracle, to fp32 reordering: per-sample relative L2 error <= 1e-4;
* an identity custom hook on a ReLU reproduces the plan's heatmaps, a doubling one gives twice
  them (every rule is linear in the incoming relevance), for compute_relevances and for
  HeatmapGenerator (K+1 replicated batch, reference explainer.py:92-104).
"""
import copy

import pytest
import torch

from lrp_common import gtzan128, logmel, ortho
from drsa_audio_amd.engine import HookedAutograd, LRPEngine, clear_cache, get_engine
from drsa_audio_amd.utils.constants import LRP_NAME_MAP_GTZAN
from drsa_audio_amd.xai.explain.attribute import compute_relevances
from drsa_audio_amd.xai.explain.explainer import HeatmapGenerator
from drsa_audio_amd.zennit.composites import NameMapComposite
from drsa_audio_amd.zennit.core import Hook

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
TOL = 1e-4


class Same(Hook):
    def backward(self, module, grad_input, grad_output):
        return grad_input


class Doubling(Hook):
    def backward(self, module, grad_input, grad_output):
        return tuple(2 * g for g in grad_input)


def _rel(a, b):
    a, b = a.double().flatten(1), b.double().flatten(1)
    return ((a - b).norm(dim=1) / b.norm(dim=1).clamp_min(1e-30)).max().item()


@pytest.fixture(scope="module")
def net():
    return gtzan128().to(DEV)


def test_routing(net):
    clear_cache()
    plain = NameMapComposite(LRP_NAME_MAP_GTZAN)
    custom = NameMapComposite(LRP_NAME_MAP_GTZAN + [(["features.1"], Doubling())])
    assert isinstance(get_engine(net, plain), LRPEngine)
    assert isinstance(get_engine(net, custom), HookedAutograd)


def test_builtin_rules_match_plan(net):
    x = logmel(4, seed=5).to(DEV)
    comp = NameMapComposite(LRP_NAME_MAP_GTZAN)
    R_plan = compute_relevances(net, x, comp, class_idx=2)
    slow = HookedAutograd(net, comp)
    slow.forward(x)
    R_slow = slow.backward(cls=torch.full((4,), 2, device=DEV, dtype=torch.int32))
    assert _rel(R_slow, R_plan) <= TOL


@pytest.mark.parametrize("hook,scale", [(Same(), 1.0), (Doubling(), 2.0)])
def test_custom_hook_compute_relevances(net, hook, scale):
    x = logmel(4, seed=6).to(DEV)
    R_plan = compute_relevances(net, x, NameMapComposite(LRP_NAME_MAP_GTZAN), class_idx=5)
    comp = NameMapComposite(LRP_NAME_MAP_GTZAN + [(["features.4"], hook)])
    R = compute_relevances(net, x, comp, class_idx=5)
    assert _rel(R, scale * R_plan) <= TOL


def test_custom_hook_heatmap_generator(net):
    U = torch.from_numpy(ortho(64, 3)).float()
    x = logmel(3, seed=7).to(DEV)
    hg = HeatmapGenerator(net, U, LRP_NAME_MAP_GTZAN, "blues", num_concepts=4, layer_idx=7, device=DEV)
    hg.generate_subspace_heatmaps(x, to_host=False)
    ref = {k: v.clone() for k, v in hg.info_device.items()}
    hg2 = HeatmapGenerator(net, U, LRP_NAME_MAP_GTZAN + [(["features.1"], Doubling())], "blues", num_concepts=4,
                           layer_idx=7, device=DEV)
    assert isinstance(get_engine(hg2.projectionmodel, hg2.composite), HookedAutograd)
    hg2.generate_subspace_heatmaps(x, to_host=True)
    out = hg2.info_device
    assert _rel(out["standard_heatmaps"], 2 * ref["standard_heatmaps"]) <= TOL
    # sorted per-sample subspace relevances and the heatmaps in that order
    assert _rel(out["subspace_relevances"], 2 * ref["subspace_relevances"]) <= TOL
    assert _rel(out["subspace_heatmaps"], 2 * ref["subspace_heatmaps"]) <= TOL
    assert hg2.info["subspace_heatmaps"].shape == (3, 4, 128, 128)


def test_slow_path_refuses_host_input(net):
    from drsa_audio_amd import _capi
    comp = NameMapComposite(LRP_NAME_MAP_GTZAN + [(["features.1"], Doubling())])
    with pytest.raises(_capi.DrsaAmdError):
        compute_relevances(net, logmel(1), comp, class_idx=0)
