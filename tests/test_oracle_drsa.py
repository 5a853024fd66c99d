"""The DRSA oracle (oracle/drsa_ref.py) against golden vectors produced by the REFERENCE
drsa.py (oracle/gen_fixtures.py), plus the closed-form gradient the HIP kernel uses."""
import os

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


# ---------------------------------------------------------------------------------------------
# round-2 fixtures: long-horizon reference runs (C3 2000 steps, C4 shape, d=100) and drsa.main
# ---------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def lfx(golden_dir):
    return np.load(f"{golden_dir}/drsa_long_fixture.npz")


@pytest.mark.parametrize("tag", ["c3", "c4", "d100"])
def test_long_inputs_regenerate(lfx, tag):
    N, d, K, seed, _ = lfx[f"{tag}_meta"]
    A, C = drsa_inputs(N, d, seed)
    assert np.allclose([A.sum(dtype=np.float64), C.sum(dtype=np.float64)], lfx[f"{tag}_A_checksum"], rtol=0, atol=1e-6)
    if tag != "d100":   # C3 / C4 start from the bench's U (drsa.main's draw, drsa.py:265-272)
        assert np.array_equal(lfx[f"{tag}_U0"], np.load(f"{os.path.dirname(__file__)}/golden/u64_seed42.npy"))


def test_oracle_c4_trajectory_matches_reference(lfx):
    """The op-for-op oracle against the reference's own 10-step run at the C4 shape (N=160000, K=8)."""
    N, d, K, seed, steps = lfx["c4_meta"]
    A, C = map(torch.from_numpy, drsa_inputs(N, d, seed))
    U, traj = drsa_ref.run(A, C, torch.from_numpy(lfx["c4_U0"]), int(K), int(steps))
    np.testing.assert_allclose(np.array(traj), lfx["c4_traj"], rtol=1e-6, atol=0)
    assert np.abs(U.numpy() - lfx["c4_Ufinal"]).max() < 1e-5


@pytest.mark.parametrize("tag,n", [("c3", 300), ("d100", 120)])
def test_float64_closed_form_tracks_reference_long_horizon(lfx, tag, n):
    """Reference fp32 steps with fp64 eigh vs the float64 closed form with an exact polar factor.
    Over the whole horizon (2000 C3 / 500 d=100 steps) the trajectories stay within 3.6e-7 /
    3.2e-7 relative (measured once, ~80 s); the CPU suite replays the first n steps.  The dynamics
    are contractive, so an fp32 device implementation has the 1e-4 budget to spare
    (tests/test_drsa_long_gpu.py runs the full horizon on the GPU)."""
    N, d, K, seed, steps = lfx[f"{tag}_meta"]
    A, C = drsa_inputs(N, d, seed)
    U = lfx[f"{tag}_U0"].astype(np.float64)
    traj = []
    for _ in range(n):
        f, G, _, _ = drsa_ref.closed_form(A, C, U, int(K))
        traj.append(f)
        U = drsa_ref.polar(U + G)
    ref = lfx[f"{tag}_traj"][:n]
    assert np.max(np.abs(np.array(traj) - ref) / np.abs(ref)) < 1e-6


def test_oracle_main_schedule_and_runs_match_reference(lfx):
    """drsa.main (drsa.py:241-301) end to end: 3 runs from compounding permutations of one
    ortho_group draw; every run's trajectory and final U equal the reference's bit for bit."""
    N, d, K, seed, steps, runs, rseed = (int(v) for v in lfx["main_meta"])
    A, C = map(torch.from_numpy, drsa_inputs(N, d, seed))
    for r, U0 in enumerate(drsa_ref.initial_us(d, runs, rseed)):
        U, traj = drsa_ref.run(A, C, torch.from_numpy(U0), K, steps)
        np.testing.assert_allclose(np.array(traj), lfx["main_traj"][r], rtol=1e-6, atol=0)
        assert np.abs(U.numpy() - lfx["main_Ufinal"][r]).max() < 1e-5


def _embed(d, K):
    """The padded embedding the HIP kernels use for any d (csrc/drsa_step.hip: geom/pad_col)."""
    dk = d // K
    DKp = 1 << (dk - 1).bit_length()
    DP = 1 << (max(16, K * DKp) - 1).bit_length()
    cols = np.array([(j // dk) * DKp + j % dk for j in range(d)])
    padcols = np.array(sorted(set(range(DP)) - set(cols.tolist())))
    return DP, DKp, cols, padcols


@pytest.mark.parametrize("d,K", [(100, 4), (48, 4), (100, 25), (96, 6), (12, 3)])
def test_padded_embedding_is_exact(d, K):
    """Objective, gradient and polar factor of the padded problem equal the real problem's
    (float64): zero padding of A, C, U, concept blocks moved to power-of-two slots, and an
    identity block pairing padded rows with padded columns in the polar step."""
    rng = np.random.default_rng(d + K)
    N = 500
    A = np.abs(rng.standard_normal((N, d)))
    C = rng.standard_normal((N, d))
    U = np.linalg.qr(rng.standard_normal((d, d)))[0]
    DP, DKp, cols, padcols = _embed(d, K)
    Ap = np.zeros((N, DP)); Ap[:, :d] = A
    Cp = np.zeros((N, DP)); Cp[:, :d] = C
    Up = np.zeros((DP, DP)); Up[np.ix_(np.arange(d), cols)] = U
    f, G, _, _ = drsa_ref.closed_form(A, C, U, K)
    # padded problem with Kp = DP/DKp concept slots; the phantom ones are all-zero columns
    Kp = DP // DKp
    XA, XC = Ap @ Up, Cp @ Up
    s = (XA * XC).reshape(N, Kp, DKp).sum(-1)
    r = np.maximum(s, 0)
    S = (r * r).sum(0)
    assert np.all(S[K:] == 0)
    M = np.sqrt(S[:K] / N)
    fp = float(np.mean(np.sqrt(M)) ** 2)
    c = np.concatenate([np.sqrt(fp) / (K * N * M ** 1.5), np.zeros(Kp - K)])
    Gp = Ap.T @ (np.repeat(r, DKp, axis=1) * XC) + Cp.T @ (np.repeat(r, DKp, axis=1) * XA)
    Gp = Gp * np.repeat(c, DKp)[None, :]
    assert abs(fp - f) <= 1e-14 * f
    np.testing.assert_allclose(Gp[np.ix_(np.arange(d), cols)], G, rtol=0, atol=1e-13 * np.abs(G).max())
    assert np.abs(Gp[d:]).max() == 0 and np.abs(Gp[:, padcols]).max() == 0
    Vp = Up + Gp
    Vp[np.arange(d, DP), padcols] = 1.0
    Pp = drsa_ref.polar(Vp)
    np.testing.assert_allclose(Pp[np.ix_(np.arange(d), cols)], drsa_ref.polar(U + G), atol=1e-12)
