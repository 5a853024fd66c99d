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
