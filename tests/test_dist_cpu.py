"""Multi-process (world_size 2, gloo, CPU) test of the row-sharded DRSA orchestration.

The per-step kernels are replaced by the oracle's float64 closed form (the HIP kernels need a
GPU); what is tested here is the distributed logic: global row count, one all-reduce of the
[d*d + K] partial per step, every rank ending with identical U and trajectory, equal to the
unsharded run."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class OracleBackend:
    def __init__(self, A, C, d, K):
        self.A, self.C, self.d, self.K = A.double().numpy(), C.double().numpy(), d, K

    def slab_size(self):
        return self.d * self.d + self.K

    def partial(self, U):
        Ud = U.double().numpy()
        XA, XC = self.A @ Ud, self.C @ Ud
        N = self.A.shape[0]
        s = (XA * XC).reshape(N, self.K, -1).sum(-1)
        r = np.maximum(s, 0)
        R = np.repeat(r, self.d // self.K, axis=1)
        G = self.A.T @ (R * XC) + self.C.T @ (R * XA)
        return torch.from_numpy(np.concatenate([G.reshape(-1), (r * r).sum(0)]))

    def _scal(self, gs, N):
        S = gs[self.d * self.d:].numpy()
        M = np.sqrt(S / N)
        f = float(np.mean(np.sqrt(M)) ** 2)
        return f, M

    def finish(self, gs, N, U):
        import drsa_ref
        f, M = self._scal(gs, N)
        c = np.sqrt(f) / (self.K * N * M ** 1.5)
        G = gs[:self.d * self.d].numpy().reshape(self.d, self.d) * np.repeat(c, self.d // self.K)[None, :]
        Un = drsa_ref.polar(U.double().numpy() + G)
        return torch.from_numpy(Un), torch.tensor([f], dtype=torch.float64)

    def objective(self, gs, N, U):
        return torch.tensor([self._scal(gs, N)[0]], dtype=torch.float64)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, A, C, U0, K, steps, q):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from drsa_audio_amd.xai.drsa.distributed import shard_rows, sharded_run
    sl = shard_rows(A.size(0), world, rank)
    be = OracleBackend(A[sl], C[sl], U0.size(0), K)
    U, traj = sharded_run(A[sl], C[sl], U0.double(), K, steps, backend=be)
    q.put((rank, U.numpy(), traj))
    dist.destroy_process_group()


def test_sharded_drsa_two_ranks_matches_unsharded():
    import drsa_ref
    from gen_fixtures import drsa_inputs
    A, C = (torch.from_numpy(v) for v in drsa_inputs(999, 16, 4))
    U0 = torch.from_numpy(np.linalg.qr(np.random.default_rng(1).standard_normal((16, 16)))[0])
    K, steps = 4, 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, A, C, U0, K, steps, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: (u, t) for r, u, t in (q.get(timeout=120) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.array_equal(res[0][0], res[1][0]) and np.array_equal(res[0][1], res[1][1])
    # unsharded float64 reference trajectory
    U = U0.numpy()
    ref = []
    for _ in range(steps):
        f, G, _, _ = drsa_ref.closed_form(A.numpy(), C.numpy(), U, K)
        ref.append(f)
        U = drsa_ref.polar(U + G)
    ref.append(drsa_ref.closed_form(A.numpy(), C.numpy(), U, K)[0])
    assert np.allclose(res[0][1], ref, rtol=1e-12, atol=0), (res[0][1], ref)
    assert np.abs(res[0][0] - U).max() < 1e-10


def _worker_joint(rank, world, port, probs, steps, q):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from drsa_audio_amd.xai.drsa.distributed import shard_rows, sharded_run_joint
    local, bes = [], []
    for A, C, U0, K in probs:
        sl = shard_rows(A.size(0), world, rank)
        local.append((A[sl], C[sl], U0.double(), K))
        bes.append(OracleBackend(A[sl], C[sl], U0.size(0), K))
    out = sharded_run_joint(local, steps, backends=bes)
    q.put((rank, [(u.numpy(), t) for u, t in out]))
    dist.destroy_process_group()


def test_joint_two_problem_sharded_matches_separate_unsharded():
    """C5-style joint optimisation of two layers (different d and K) over 2 ranks with one
    all-reduce per step equals each problem optimised alone."""
    import drsa_ref
    from gen_fixtures import drsa_inputs
    probs = []
    for (N, d, K, seed) in ((301, 16, 4, 1), (257, 32, 8, 2)):
        A, C = (torch.from_numpy(v) for v in drsa_inputs(N, d, seed))
        U0 = torch.from_numpy(np.linalg.qr(np.random.default_rng(seed).standard_normal((d, d)))[0])
        probs.append((A, C, U0, K))
    steps = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_joint, args=(r, 2, port, probs, steps, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for pi, (A, C, U0, K) in enumerate(probs):
        U = U0.numpy()
        ref = []
        for _ in range(steps):
            f, G, _, _ = drsa_ref.closed_form(A.numpy(), C.numpy(), U, K)
            ref.append(f)
            U = drsa_ref.polar(U + G)
        ref.append(drsa_ref.closed_form(A.numpy(), C.numpy(), U, K)[0])
        for r in (0, 1):
            assert np.allclose(res[r][pi][1], ref, rtol=1e-12, atol=0)
            assert np.abs(res[r][pi][0] - U).max() < 1e-10


def test_shard_rows_partition():
    from drsa_audio_amd.xai.drsa.distributed import shard_rows
    for N in (0, 1, 7, 160000):
        for world in (1, 2, 3, 8):
            parts = [shard_rows(N, world, r) for r in range(world)]
            assert parts[0].start == 0 and parts[-1].stop == N
            assert all(parts[i].stop == parts[i + 1].start for i in range(world - 1))
            sizes = [p.stop - p.start for p in parts]
            assert max(sizes) - min(sizes) <= 1


# ---------------------------------------------------------------- task-parallel DRSA grid
def _oracle_runner(problems, steps):
    """float64 closed-form DRSA run per problem (drsa_ref), in the product runner's contract."""
    import drsa_ref
    out = []
    for A, C, U0, K in problems:
        A_, C_, U = A.double().numpy(), C.double().numpy(), U0.double().numpy()
        traj = []
        for _ in range(steps):
            f, G, _, _ = drsa_ref.closed_form(A_, C_, U, K)
            traj.append(f)
            U = drsa_ref.polar(U + G)
        traj.append(drsa_ref.closed_form(A_, C_, U, K)[0])
        out.append((torch.from_numpy(U), np.asarray(traj)))
    return out


def _grid_data():
    from gen_fixtures import drsa_inputs
    data = {}
    for ci, c in enumerate(("pop", "metal", "disco")):
        for l, d in ((19, 12), (26, 16)):
            A, C = drsa_inputs(60 + 7 * ci + l, d, 10 * ci + l)
            data[(c, l)] = (torch.from_numpy(A), torch.from_numpy(C))
    return data


def _worker_grid(rank, world, port, root, steps, q):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from drsa_audio_amd.xai.drsa.cluster.optsubspaces import optimize_grid
    res = optimize_grid(_grid_data(), root, num_concepts=4, steps=steps, runs=3, runner=_oracle_runner)
    q.put((rank, {k: (v["objective"], v["rank"]) for k, v in res.items()}))
    dist.destroy_process_group()


def test_assign_lpt_balanced_and_deterministic():
    from drsa_audio_amd.xai.drsa.cluster.optsubspaces import GTZAN_CLASSES, assign, problem_grid
    shapes = {(c, l): (20000, d) for c in GTZAN_CLASSES for l, d in ((19, 100), (26, 128), (33, 128))}
    tasks = problem_grid(shapes, 3)
    assert len(tasks) == 90 and len({t.key for t in tasks}) == 90
    for world in (1, 2, 4, 8):
        parts = assign(tasks, world)
        assert sorted(t.key for p in parts for t in p) == sorted(t.key for t in tasks)
        sizes = [len(p) for p in parts]
        assert max(sizes) - min(sizes) <= 1          # d=100 pads to 128: equal costs
        assert parts == assign(tasks, world)


def test_task_parallel_grid_two_ranks_matches_sequential(tmp_path):
    """optsubspaces grid over 2 gloo ranks: every (class, layer, run) problem equals the
    sequential drsa.main schedule (same initial U per run), files as drsa.main writes them."""
    import pickle
    import pandas as pd
    from drsa_audio_amd.xai.drsa.drsa import initial_projections
    steps = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    root = str(tmp_path / "models")
    procs = [ctx.Process(target=_worker_grid, args=(r, 2, port, root, steps, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == res[1] and len(res[0]) == 18
    assert {r for _, r in res[0].values()} == {0, 1}
    data = _grid_data()
    for (c, l), (A, C) in data.items():
        U0s = initial_projections(A.size(1), 3, 42)
        for run in (1, 2, 3):
            (U_ref, tr_ref), = _oracle_runner([(A, C, torch.tensor(U0s[run - 1], dtype=torch.float32), 4)], steps)
            path = os.path.join(root, c, f"layer{l}", f"run{run}")
            with open(os.path.join(path, "projection_matrix.pkl"), "rb") as fh:
                U = pickle.load(fh)               # our own file (float32 numpy), written by this test
            tr = pd.read_csv(os.path.join(path, "train_stats.csv"))["loss"].to_numpy()
            assert U.dtype == np.float32 and np.array_equal(U, U_ref.numpy().astype(np.float32))
            assert len(tr) == steps + 1 and np.allclose(tr, tr_ref, rtol=1e-6)
            assert res[0][(c, l, run)][0] == float(tr_ref[-1])


def test_launcher_spawns_ranks_and_forwards_rank0(tmp_path):
    """utils/launch.spawn: N ranks with the torchrun environment, rank 0's stdout forwarded, a
    failing rank's exit code returned."""
    import subprocess
    import sys
    script = tmp_path / "w.py"
    script.write_text(
        "import os, sys\n"
        f"sys.path.insert(0, {ROOT!r})\n"
        "from drsa_audio_amd.utils.launch import maybe_launch, init_distributed\n"
        "maybe_launch(int(sys.argv[1]), one_device=True)\n"
        "import torch, torch.distributed as dist\n"
        "world, rank, dev = init_distributed('gloo', one_device=True)\n"
        "t = torch.tensor([rank + 1.0]); dist.all_reduce(t)\n"
        "if rank == 0: print('SUM', world, float(t))\n"
        "dist.destroy_process_group()\n"
        "sys.exit(3 if len(sys.argv) > 2 and rank == 1 else 0)\n")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, str(script), "3"], env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip().splitlines()[-1] == "SUM 3 6.0"   # (gloo logs its connections to stdout)
    r = subprocess.run([sys.executable, str(script), "2", "fail"], env=env, capture_output=True, text=True,
                       timeout=180)
    assert r.returncode == 3


class OracleNormOps:
    """normalize_vectors' two halves in numpy (the HIP kernels need a GPU): fp64 sum of squares,
    then v / fl32(sqrt(sum / n)) / fl32(d^(1/4)) as preprocessing.py:229-231 writes it."""

    def sumsq(self, v):
        return torch.tensor([float(np.sum(v.double().numpy() ** 2))], dtype=torch.float64)

    def scale(self, v, sums, n_total, out):
        s = 0.0
        for x in sums.tolist():          # rank order
            s += x
        E = np.float32(np.sqrt(s / n_total))
        d4 = np.float32(v.size(-1) ** 0.25)
        out.copy_(torch.from_numpy(v.numpy() / E / d4))


def _worker_norm(rank, world, port, sizes, V, q):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from drsa_audio_amd.xai.drsa.preprocessing import _sample_offset, normalize_vectors
    lo = sum(sizes[:rank])
    local = V[lo:lo + sizes[rank]].clone()
    out = normalize_vectors(local, group=dist.group.WORLD, _ops=OracleNormOps())
    off = _sample_offset(sizes[rank] // 4, dist.group.WORLD)
    q.put((rank, out.numpy(), off))
    dist.destroy_process_group()


@pytest.mark.parametrize("sizes", [(600, 400), (1000, 0)])
def test_normalize_vectors_two_ranks_equals_single_process(sizes):
    """normalize_vectors(group=...) on row shards equals the single-process normalisation of the
    concatenation (getdrsadata.py:47-59 normalises the whole set): every rank's rows, bit for bit;
    a rank without rows contributes nothing; the sample offsets are the ranks' prefix sums."""
    rng = np.random.default_rng(5)
    V = torch.from_numpy((rng.standard_normal((sum(sizes), 16)) * 3).astype(np.float32))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_norm, args=(r, 2, port, list(sizes), V, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: (o, off) for r, o, off in (q.get(timeout=120) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ops = OracleNormOps()
    ref = torch.empty_like(V)
    ops.scale(V, ops.sumsq(V), V.numel(), ref)
    got = np.concatenate([res[0][0], res[1][0]])
    assert np.array_equal(got, ref.numpy())
    assert res[0][1] == (0, sum(sizes) // 4) and res[1][1] == (sizes[0] // 4, sum(sizes) // 4)
