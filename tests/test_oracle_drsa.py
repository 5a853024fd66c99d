"""The DRSA oracle (oracle/drsa_ref.py) against golden vectors produced by the REFERENCE
drsa.py (oracle/gen_fixtures.py), plus the closed-form gradient the HIP kernel uses."""
import numpy as np
import pytest
import torch

import drsa_ref
from gen_fixtures import drsa_inputs


@pytest.fixture(scope="module")
def fx(golden_dir):
    return np.load(f"{golden_dir}/drsa_fixture.npz")


def test_fmean_objective(fx):
    X = torch.from_numpy(fx["fmean_in"])
    assert np.array_equal(drsa_ref.generalized_fmean(X, 2).numpy(), fx["fmean_p2"])
    assert np.array_equal(drsa_ref.generalized_fmean(X, 0.5).numpy(), fx["fmean_p05"])
    assert np.array_equal(drsa_ref.objective_fn(X).numpy(), fx["objective"])


@pytest.mark.parametrize("tag", ["small", "c3w"])
def test_inputs_regenerate(fx, tag):
    N, d, K, seed, _ = fx[f"{tag}_meta"]
    A, C = drsa_inputs(N, d, seed)
    assert np.allclose([A.sum(dtype=np.float64), C.sum(dtype=np.float64)], fx[f"{tag}_A_checksum"], rtol=0, atol=1e-9)


@pytest.mark.parametrize("tag", ["small", "c3w"])
def test_oracle_step_and_trajectory_bit_exact(fx, tag):
    N, d, K, seed, steps = fx[f"{tag}_meta"]
    A, C = map(torch.from_numpy, drsa_inputs(N, d, seed))
    U0 = torch.from_numpy(fx[f"{tag}_U0"])
    U1, f0, G0 = drsa_ref.step(A, C, U0, K)
    assert f0 == float(fx[f"{tag}_f0"])
    assert np.array_equal(G0.numpy(), fx[f"{tag}_G0"])
    assert np.array_equal(U1.numpy(), fx[f"{tag}_orth0"])
    U, traj = drsa_ref.run(A, C, U0, K, int(steps))
    assert np.array_equal(np.array(traj, dtype=np.float64), fx[f"{tag}_traj"])
    assert np.array_equal(U.numpy(), fx[f"{tag}_Ufinal"])


@pytest.mark.parametrize("tag", ["small", "c3w"])
def test_closed_form_gradient_matches_autograd(fx, tag):
    N, d, K, seed, _ = fx[f"{tag}_meta"]
    A, C = drsa_inputs(N, d, seed)
    f, G, _, _ = drsa_ref.closed_form(A, C, fx[f"{tag}_U0"], K)
    assert abs(f - float(fx[f"{tag}_f0"])) <= 1e-6 * abs(f)
    assert np.abs(G - fx[f"{tag}_G0"]).max() <= 1e-5 * np.abs(G).max()
    # and in float64 against float64 autograd
    A64, C64, U64 = (torch.from_numpy(np.asarray(v, dtype=np.float64)) for v in (A, C, fx[f"{tag}_U0"]))
    Ug = U64.clone().requires_grad_(True)
    x = ((A64 @ Ug) * (C64 @ Ug)).view(-1, K, d // K).sum(-1).relu()
    obj = torch.pow(torch.mean(torch.pow(torch.pow(torch.mean(x ** 2, 0), 0.5), 0.5), 0), 2)
    obj.backward()
    assert np.abs(Ug.grad.numpy() - G).max() <= 1e-12 * max(1.0, np.abs(G).max())


def test_main_initial_u_schedule(fx):
    assert np.array_equal(np.stack(drsa_ref.initial_us(16, 3, 42)), fx["main_U_runs"])


def test_polar_matches_orthogonalize(fx):
    V = fx["small_U0"] + fx["small_G0"]
    P = drsa_ref.polar(V)
    assert np.abs(P - fx["small_orth0"]).max() < 1e-5


def test_bf16_round_matches_torch():
    """oracle bf16 rounding (used by the bf16-path closed form) = torch's float32->bfloat16 (RNE)."""
    import torch
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.standard_normal(10000).astype(np.float32) * 10 ** rng.uniform(-5, 5, 10000).astype(np.float32),
                        np.array([0.0, -0.0, 1.0, 1.00390625, 1.01171875, 3.0e-39], dtype=np.float32)])
    ref = torch.from_numpy(x).to(torch.bfloat16).float().numpy()
    assert np.array_equal(drsa_ref.bf16_round(x), ref)
