"""VGGish-BN (C5 model) through the HIP engine vs the exact-order oracle (GPU).

Covers what GTZAN-128 does not: block_depth 2 (conv stages without a pool), BatchNorm merged by
SequentialMergeBatchNorm (trunk and head), a (2,4) max-pool, 100-channel layers (padded to 128),
128x128 convs, and DRSA data capture at the C5 layers j = 26 and j = 33 (d = 128).
Parity: bit-identical to lrp_ref mode="exact" on the merged model (oracle.merge_batch_norm
restates zennit's canonizer).
"""
import numpy as np
import pytest
import torch

import drsa_ref
import lrp_ref
from lrp_common import logmel, ortho, spec, vggish
from drsa_audio_amd.utils.constants import LRP_NAME_MAP_VGGISH
from drsa_audio_amd.zennit.canonizers import SequentialMergeBatchNorm
from drsa_audio_amd.zennit.composites import NameMapComposite

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _comp():
    return NameMapComposite(LRP_NAME_MAP_VGGISH, canonizers=[SequentialMergeBatchNorm()])


@pytest.fixture(scope="module")
def small():
    return vggish(input_size=(64, 128))   # smallest conv map 4x4 (W % 4 == 0)


def test_vggish_small_standard_lrp_bit_exact(small):
    from drsa_audio_amd.xai.explain.attribute import compute_relevances
    import copy
    x = logmel(3, 64, 128, seed=3)
    _, R = lrp_ref.lrp(lrp_ref.merge_batch_norm(small), spec(LRP_NAME_MAP_VGGISH), x, class_idx=4, mode="exact")
    Rg = compute_relevances(copy.deepcopy(small).to(DEV), x.to(DEV), _comp(), class_idx=4)
    assert Rg.shape == x.shape
    assert torch.equal(Rg.cpu(), R)


def test_vggish_full_size_standard_lrp_bit_exact():
    from drsa_audio_amd.xai.explain.attribute import compute_relevances
    net = vggish()
    x = logmel(1, 128, 256, seed=5)
    _, R = lrp_ref.lrp(lrp_ref.merge_batch_norm(net), spec(LRP_NAME_MAP_VGGISH), x, class_idx=2, mode="exact")
    Rg = compute_relevances(net.to(DEV), x.to(DEV), _comp(), class_idx=2)
    assert torch.equal(Rg.cpu(), R)


@pytest.mark.parametrize("layer_idx", [26, 33, 19, 20])
def test_vggish_drsa_capture_bit_exact(small, layer_idx):
    from drsa_audio_amd.xai.drsa.preprocessing import get_intermediate, preprocess_data
    import copy
    x = logmel(2, 64, 128, seed=layer_idx)
    _, _, (act, rel) = lrp_ref.lrp(lrp_ref.merge_batch_norm(small), spec(LRP_NAME_MAP_VGGISH), x, class_idx=1,
                                   mode="exact", capture=f"features.{layer_idx}")
    m = copy.deepcopy(small).to(DEV)
    a, r = get_intermediate(m, x.to(DEV), _comp(), layer_idx, 1)
    assert torch.equal(a.cpu(), act) and torch.equal(r.cpu(), rel)
    L = min(4, act.shape[-1] * act.shape[-2])
    np.random.seed(5)
    idx = drsa_ref.sample_spatial_locations(2, act.shape[-2:], L)
    va = drsa_ref.get_vectors_from_maps(act, idx)
    ctx = drsa_ref.compute_context_vectors(va, drsa_ref.get_vectors_from_maps(rel, idx))
    np.random.seed(5)
    A, C = preprocess_data(m, x.to(DEV), _comp(), layer_idx, 1, num_locations=L)
    assert torch.equal(A.cpu(), va) and torch.equal(C.cpu(), ctx)


def test_vggish_capture_at_wide_pool_layer(small):
    """capture at the ReLU before the (2,4) pool (features.5): relevance arrives through the
    2x4 argmax."""
    from drsa_audio_amd.xai.drsa.preprocessing import get_intermediate
    import copy
    x = logmel(2, 64, 128, seed=11)
    _, _, (act, rel) = lrp_ref.lrp(lrp_ref.merge_batch_norm(small), spec(LRP_NAME_MAP_VGGISH), x, class_idx=0,
                                   mode="exact", capture="features.5")
    a, r = get_intermediate(copy.deepcopy(small).to(DEV), x.to(DEV), _comp(), 5, 0)
    assert torch.equal(a.cpu(), act) and torch.equal(r.cpu(), rel)


@pytest.mark.parametrize("layer_idx", [19, 16])
def test_vggish_d100_heatmap_generator_bit_exact(small, layer_idx):
    """d = 100 projection (j = 19: 2x2 pool after it; j = 16: a conv after it, a' is the stage
    output) fanned out to K+1 = 5 clones, bit-identical to the exact oracle on the merged model."""
    import copy
    from drsa_audio_amd.model.modify_model import ProjectionModel
    from drsa_audio_amd.xai.explain.explainer import HeatmapGenerator
    U = ortho(100, 7 + layer_idx)
    x = logmel(2, 64, 128, seed=40 + layer_idx)
    pm = ProjectionModel(lrp_ref.merge_batch_norm(small), layer_idx, U, 4).eval()
    ref = lrp_ref.subspace_heatmaps(pm, spec(LRP_NAME_MAP_VGGISH), 4, x, class_idx=2, mode="exact")
    hg = HeatmapGenerator(copy.deepcopy(small).to(DEV), U, LRP_NAME_MAP_VGGISH, "disco", num_concepts=4,
                          layer_idx=layer_idx, device="cuda", canonizers=[SequentialMergeBatchNorm()])
    hg.generate_subspace_heatmaps(x)
    for k in ("standard_heatmaps", "standard_relevance", "subspace_heatmaps", "subspace_relevances", "mask"):
        assert np.array_equal(hg.info[k], ref[k]), k
    # the K subspace heatmaps sum to the standard one (up to fp32 rounding of the sum)
    np.testing.assert_allclose(hg.info["subspace_heatmaps"].sum(1), hg.info["standard_heatmaps"][:, 0],
                               rtol=1e-3, atol=1e-6 * np.abs(hg.info["standard_heatmaps"]).max())
