"""compute_subspace_relevances (R11, reference cxai/xai/explain/explainer.py:206-242).

Fixture: tests/golden/subspace_rel_fixture.npz, produced by executing the REFERENCE function
(extracted from explainer.py's source, oracle/gen_fixtures.py::_subspace_relevances) on the
SUBREL_CASES inputs, which regenerate from their seeds here.

* CPU: the oracle restatement (oracle/lrp_ref.py) equals the reference output bit for bit.
* GPU: drsa_amd_subspace_relevances within the BASELINE tolerance: |r - r_ref| <= 1e-4 * max_k |r_ref|
  per instance (relative to the instance's largest concept relevance: single concepts can sum
  to ~0 by cancellation), and within the same bound of a float64 evaluation.
"""
import numpy as np
import pytest
import torch

import lrp_ref
from gen_fixtures import SUBREL_CASES, subrel_inputs


@pytest.fixture(scope="module")
def sfx(golden_dir):
    return np.load(f"{golden_dir}/subspace_rel_fixture.npz")


def _f64(act, ctx, U, K):
    a = act if act.ndim == 3 else act[None]
    c = ctx if ctx.ndim == 3 else ctx[None]
    x = (a.astype(np.float64) @ U.astype(np.float64)) * (c.astype(np.float64) @ U.astype(np.float64))
    b, N, d = x.shape
    return x.reshape(b, N, K, d // K).sum(axis=(1, 3))


@pytest.mark.parametrize("i", range(len(SUBREL_CASES)))
def test_oracle_matches_reference_fixture(sfx, i):
    b, N, d, K, seed = SUBREL_CASES[i]
    assert list(sfx[f"case{i}_meta"]) == [b, N, d, K, seed]
    act, ctx, U = subrel_inputs(b, N, d, seed)
    np.testing.assert_allclose([act.sum(dtype=np.float64), ctx.sum(dtype=np.float64), U.sum(dtype=np.float64)],
                               sfx[f"case{i}_checksum"], rtol=0, atol=1e-6)
    r = lrp_ref.compute_subspace_relevances(torch.from_numpy(act), torch.from_numpy(ctx), torch.from_numpy(U), K)
    assert np.array_equal(r.numpy(), sfx[f"case{i}_rel"])
    # and the float64 value is inside the tolerance the GPU test uses
    ref = sfx[f"case{i}_rel"].astype(np.float64)
    assert np.all(np.abs(_f64(act, ctx, U, K) - ref) <= 1e-4 * np.abs(ref).max(axis=1, keepdims=True))


def test_refuses_cpu_and_bad_shapes():
    from drsa_audio_amd import _capi
    from drsa_audio_amd.xai.explain.explainer import compute_subspace_relevances
    a = torch.rand(2, 10, 16)
    with pytest.raises(_capi.DrsaAmdError):
        compute_subspace_relevances(a, a, torch.eye(16), 4)


@pytest.mark.gpu
@pytest.mark.parametrize("i", range(len(SUBREL_CASES)))
def test_hip_matches_reference_fixture(sfx, i):
    from drsa_audio_amd.xai.explain.explainer import compute_subspace_relevances
    b, N, d, K, seed = SUBREL_CASES[i]
    act, ctx, U = subrel_inputs(b, N, d, seed)
    dev = torch.device("cuda")
    r = compute_subspace_relevances(torch.from_numpy(act).to(dev), torch.from_numpy(ctx).to(dev),
                                    torch.from_numpy(U).to(dev), K)
    r = r.cpu().numpy().astype(np.float64)
    ref = sfx[f"case{i}_rel"].astype(np.float64)
    assert r.shape == ref.shape
    scale = np.abs(ref).max(axis=1, keepdims=True)
    assert np.all(np.abs(r - ref) <= 1e-4 * scale), np.abs(r - ref).max() / scale.min()
    assert np.all(np.abs(r - _f64(act, ctx, U, K)) <= 1e-4 * scale)


@pytest.mark.gpu
def test_hip_validation_and_determinism():
    from drsa_audio_amd.xai.explain.explainer import compute_subspace_relevances
    dev = torch.device("cuda")
    a = torch.rand(3, 500, 64, device=dev)
    c = torch.randn(3, 500, 64, device=dev)
    U = torch.randn(64, 64, device=dev)
    with pytest.raises(ValueError):
        compute_subspace_relevances(a, c[:, :400], U, 4)          # ctx shape differs from act
    with pytest.raises(ValueError):
        compute_subspace_relevances(a, c, U[:32, :32], 4)         # U not d x d
    with pytest.raises(ValueError):
        compute_subspace_relevances(a, c, U, 5)                   # K does not divide d
    with pytest.raises(Exception):
        compute_subspace_relevances(a, c.cpu(), U, 4)             # ctx on the host
    r1 = compute_subspace_relevances(a, c, U, 4)
    r2 = compute_subspace_relevances(a, c, U, 4)
    assert torch.equal(r1, r2)
    # 2-D input = a batch of one; non-contiguous input accepted like the reference
    r3 = compute_subspace_relevances(a[1], c[1], U, 4)
    assert torch.equal(r3[0], r1[1])
    r4 = compute_subspace_relevances(a.transpose(0, 1).contiguous().transpose(0, 1), c, U, 4)
    assert torch.equal(r4, r1)
