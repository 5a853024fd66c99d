"""Engine plan cache (engine/__init__.py): bounded, weakly referenced, buffers released."""
import gc

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _toy():
    from drsa_audio_amd.model.create_model import VGGType
    torch.manual_seed(0)
    return VGGType(n_filters=(8, 8, 16, 16, 16), n_dense=32, n_classes=2, pool_kernels=((2, 2),) * 5,
                   dropout=0.0, input_size=(64, 64), conv_bn=False, dense_bn=False, block_depth=1).eval()


def test_heatmap_generator_loop_keeps_memory_bounded():
    """The reference builds a HeatmapGenerator per pass (cpf.py:161); a drop-in must not grow."""
    from drsa_audio_amd import engine
    from drsa_audio_amd.utils.constants import LRP_NAME_MAP_TOY
    from drsa_audio_amd.xai.explain.explainer import HeatmapGenerator
    dev = torch.device("cuda")
    m = _toy().to(dev)
    U = torch.from_numpy(np.linalg.qr(np.random.default_rng(1).standard_normal((16, 16)))[0].astype(np.float32))
    x = torch.randn(64, 1, 64, 64, device=dev)
    engine.clear_cache()
    mem = []
    for i in range(20):
        hg = HeatmapGenerator(m, U, LRP_NAME_MAP_TOY, "class1", num_concepts=4, layer_idx=7, device=dev)
        hg.generate_subspace_heatmaps(x, to_host=False)
        del hg
        gc.collect()
        torch.cuda.synchronize()
        mem.append(torch.cuda.memory_allocated())
        assert engine.cache_size() <= 8
    # entries die with their generator: no growth after the first passes
    assert max(mem[5:]) <= mem[4] + (1 << 20), mem


def test_lru_cap_and_release():
    from drsa_audio_amd import engine
    from drsa_audio_amd.utils.constants import LRP_NAME_MAP_TOY
    from drsa_audio_amd.zennit.composites import NameMapComposite
    from drsa_audio_amd.xai.explain.attribute import compute_relevances
    dev = torch.device("cuda")
    engine.clear_cache()
    m = _toy().to(dev)
    x = torch.randn(4, 1, 64, 64, device=dev)
    comps = [NameMapComposite(LRP_NAME_MAP_TOY) for _ in range(12)]   # kept alive: only the LRU bound applies
    outs = [compute_relevances(m, x, c, class_idx=0) for c in comps]
    assert engine.cache_size() <= 8
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    del comps
    gc.collect()
    assert engine.cache_size() == 0
