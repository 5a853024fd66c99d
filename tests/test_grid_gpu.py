"""Task-parallel DRSA grid (xai/drsa/cluster/optsubspaces.py) on one GPU.

* drsa_run_batched (one launch per phase for every problem of a padded geometry; each partial
  workgroup folds whole groups of drsa_run's fixed 256-leaf row partition on chip) equals each
  problem run alone with drsa_run (the path drsa.main takes) bit for bit, for any number of
  workgroups per problem (automatic, 1, 3, 32, 256) and for every concept width (the grouped
  kernel; the per-leaf form at width 64);
* the batched d = 100 layer-19 shape agrees with the reference's own 500-step run to 1e-4
  (tests/golden/drsa_long_fixture.npz);
* optimize_grid writes drsa.main's files for every (class, layer, run), with results equal to
  drsa_run's bit for bit, whatever the task count per launch."""
import os
import pickle

import numpy as np
import pytest
import torch

from gen_fixtures import drsa_inputs

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _data():
    data = {}
    for ci, c in enumerate(("pop", "metal")):
        for l, d in ((19, 100), (26, 128), (7, 64)):
            A, C = drsa_inputs(3000 + 100 * ci + l, d, 7 * ci + l)
            data[(c, l)] = (torch.from_numpy(A), torch.from_numpy(C))
    return data


def test_batched_equals_drsa_run_any_partition():
    from drsa_audio_amd.xai.drsa.drsa import drsa_run, drsa_run_batched, initial_projections
    data = _data()
    for geom_layers in ((19, 26), (7,)):
        probs = []
        for (c, l), (A, C) in data.items():
            if l in geom_layers:
                for U0 in initial_projections(A.size(1), 2, 42):
                    probs.append((A.to(DEV), C.to(DEV), torch.tensor(np.ascontiguousarray(U0), dtype=torch.float32,
                                                                     device=DEV), 4))
        steps = 7
        s = torch.cuda.Stream(DEV)
        runs = {}
        with torch.cuda.stream(s):
            for blocks in (0, 1, 3, 32, 256):
                runs[blocks] = drsa_run_batched(probs, steps, blocks=blocks)
        torch.cuda.synchronize()
        for i, (A, C, U0, K) in enumerate(probs):
            U, t = drsa_run(A, C, U0, K, steps)
            for blocks, out in runs.items():
                Ub, tb = out[i]
                assert np.array_equal(tb.cpu().numpy(), t.cpu().numpy()), (blocks, i)
                assert torch.equal(Ub, U), (blocks, i)


@pytest.mark.parametrize("d,K,N", [(128, 2, 5000), (64, 1, 3001), (128, 16, 4099), (100, 4, 100), (32, 4, 20000)])
def test_batched_equals_drsa_run_geometries(d, K, N):
    """Every padded geometry of the batched path: concept width 64 (the per-leaf form), 8, 32, a
    problem with fewer row blocks than leaves, many rows per leaf."""
    from drsa_audio_amd.xai.drsa.drsa import drsa_run, drsa_run_batched
    probs = []
    for j in range(3):
        A, C = drsa_inputs(N + 17 * j, d, 500 + j)
        U0 = np.linalg.qr(np.random.default_rng(j).standard_normal((d, d)))[0].astype(np.float32)
        probs.append(tuple(torch.from_numpy(v).to(DEV) for v in (A, C, U0)) + (K,))
    s = torch.cuda.Stream(DEV)
    with torch.cuda.stream(s):
        out = drsa_run_batched(probs, 5, blocks=2)
    torch.cuda.synchronize()
    for (A, C, U0, K_), (Ub, tb) in zip(probs, out):
        U, t = drsa_run(A, C, U0, K_, 5)
        assert np.array_equal(tb.cpu().numpy(), t.cpu().numpy()) and torch.equal(Ub, U)


def test_batched_long_d100_vs_reference(golden_dir):
    """Four copies of the reference's d = 100, K = 4, 500-step run batched with the automatic
    partition: objective within 1e-4 of the reference at every step (drsa.py:76-120)."""
    from gen_fixtures import DRSA_LONG
    from drsa_audio_amd.xai.drsa.drsa import drsa_run_batched
    fx = np.load(os.path.join(golden_dir, "drsa_long_fixture.npz"))
    N, d, K, seed, _, steps = DRSA_LONG["d100"]
    A, C = (torch.from_numpy(v).to(DEV) for v in drsa_inputs(N, d, seed))
    U0 = torch.from_numpy(fx["d100_U0"]).to(DEV)
    s = torch.cuda.Stream(DEV)
    with torch.cuda.stream(s):
        out = drsa_run_batched([(A, C, U0, K)] * 4, steps)
    torch.cuda.synchronize()
    ref = fx["d100_traj"]
    for U, t in out:
        dev = np.abs(t.cpu().numpy().astype(np.float64) - ref) / np.abs(ref)
        assert dev.max() <= 1e-4, dev.max()


def test_optimize_grid_files_and_equality(tmp_path):
    from drsa_audio_amd.xai.drsa.cluster.optsubspaces import optimize_grid
    from drsa_audio_amd.xai.drsa.drsa import drsa_run, initial_projections
    data = _data()
    steps = 6
    res = optimize_grid(data, str(tmp_path), num_concepts=4, steps=steps, runs=3, device=DEV, max_joint=7)
    assert len(res) == 18
    for (c, l), (A, C) in data.items():
        Ag, Cg = A.to(DEV), C.to(DEV)
        for run, U0 in enumerate(initial_projections(A.size(1), 3, 42), start=1):
            U, tr = drsa_run(Ag, Cg, torch.tensor(np.ascontiguousarray(U0), dtype=torch.float32, device=DEV), 4, steps)
            got = res[(c, l, run)]
            # optimize_grid runs drsa_run's row partition: bit-equal to drsa.main's runs
            assert np.array_equal(got["trajectory"], tr.cpu().numpy())
            assert np.array_equal(got["U"], U.cpu().numpy())
            with open(os.path.join(tmp_path, c, f"layer{l}", f"run{run}", "projection_matrix.pkl"), "rb") as fh:
                assert np.array_equal(pickle.load(fh), got["U"])   # our own file
