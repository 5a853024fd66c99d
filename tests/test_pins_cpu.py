"""Pins for the zennit-free pieces of the LRP path, against outputs of the REFERENCE functions
executed in the build container (oracle/gen_fixtures.py --round3: lrp_output_modifier
attribute.py:111-160, SubspaceHook.backward attribute.py:42-60, HeatmapGenerator.sort_subspaces
explainer.py:151-176 run from their source text).  CPU side: the product's torch-level API pieces
and the oracle's restatements; the kernels are pinned by tests/test_pins_gpu.py."""
import numpy as np
import pytest
import torch

import lrp_ref
from gen_fixtures import SORT_CASES, sort_inputs

SEED_CASES = {"cls3": dict(class_idx=3), "cls0_onehot": dict(class_idx=0, one_hot_encoded=True),
              "all10": dict(num_classes=10), "all10_onehot": dict(num_classes=10, one_hot_encoded=True),
              "cls9": dict(class_idx=9)}


@pytest.fixture(scope="module")
def pins(golden_dir):
    return np.load(f"{golden_dir}/lrp_pins_fixture.npz")


def test_output_modifier_equals_reference(pins):
    from drsa_audio_amd.xai.explain.attribute import lrp_output_modifier, seed_class_indices
    logits = torch.from_numpy(pins["seed_logits"])
    for tag, kw in SEED_CASES.items():
        ref = pins[f"seed_{tag}"]
        assert np.array_equal(lrp_output_modifier(**kw)(logits).numpy(), ref), tag
        oh = kw.get("one_hot_encoded", False)
        assert np.array_equal(lrp_ref.output_seed(logits, kw.get("class_idx"), kw.get("num_classes"), oh).numpy(), ref)
        # the fused-seed class map: row b attributes class cls[b]
        cls = seed_class_indices(logits.size(0), kw.get("class_idx"), kw.get("num_classes")).numpy()
        onehot = np.eye(10, dtype=np.float32)[cls]
        assert np.array_equal(onehot if oh else logits.numpy() * onehot, ref)
    assert int(pins["seed_all10_b16_raises"]) == 1             # D8: the reference raises at B % C != 0
    with pytest.raises(ValueError):
        lrp_output_modifier(num_classes=10)(logits[:16])
    with pytest.raises(ValueError):
        seed_class_indices(16, None, 10)


def test_subspace_hook_equals_reference(pins):
    from drsa_audio_amd.xai.explain.attribute import SubspaceHook
    for tag in ("k4", "k2", "k8", "k5"):
        g, ref = pins[f"hook_{tag}_in"], pins[f"hook_{tag}_out"]
        K = g.shape[2]
        out, = SubspaceHook(K).backward(None, None, (torch.from_numpy(g.copy()),))
        assert np.array_equal(out.numpy(), ref), tag
        assert np.array_equal(lrp_ref.subspace_mask(torch.from_numpy(g), K).numpy(), ref), tag


@pytest.mark.parametrize("ops", [lrp_ref.TorchOps, lrp_ref.ExactOps])
def test_oracle_sort_equals_reference(pins, ops):
    for i, (B, K, H, W, seed) in enumerate(SORT_CASES):
        hm = sort_inputs(B, K, H, W, seed)
        assert hm.sum(dtype=np.float64) == pins[f"sort{i}_checksum"][0]
        sub_s, rel, mask = lrp_ref.sort_subspaces(hm[:, 1:], ops)
        assert np.array_equal(mask, pins[f"sort{i}_mask"]), i
        assert np.array_equal(rel, pins[f"sort{i}_rel"]), i
        assert np.array_equal(sub_s, hm[:, 1:][np.arange(B)[:, None], pins[f"sort{i}_mask"]])
        assert np.array_equal(ops.plane_sum(hm[:, 0:1]).flatten(), pins[f"sort{i}_std_rel"]), i
    assert int(pins["sort_b1_raises"]) == 1                   # D7: the reference fails at B = 1


def test_numpy_pairwise_restatement():
    """The summation order the heatmap_sort kernels implement, restated, equals numpy's float32
    sum for the balanced, serial-walk, single-leaf, tail and n < 8 cases."""
    rng = np.random.default_rng(3)
    for n in (4, 7, 8, 36, 64, 128, 136, 256, 1872, 4096, 1000, 8192, 10000, 16384, 20000, 32768):
        x = (rng.standard_normal(n) * np.exp(rng.standard_normal(n) * 2)).astype(np.float32)
        assert lrp_ref.numpy_pairwise_sum(x) == x.reshape(1, -1).sum(axis=-1)[0], n
