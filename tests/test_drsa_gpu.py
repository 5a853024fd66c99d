"""DRSA HIP path vs the oracle / reference fixtures (GPU).

Tolerances (BASELINE.json): DRSA objective within 1e-4 relative; we test the single step
tighter (1e-5) and the 10-step trajectory against the reference's own trajectory at 1e-4.
"""
import os

import numpy as np
import pytest
import torch

import drsa_ref
from gen_fixtures import drsa_inputs

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda")


def _gpu(*arrs):
    return [torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(DEV) for a in arrs]


@pytest.fixture(scope="module")
def fx(golden_dir):
    return np.load(f"{golden_dir}/drsa_fixture.npz")


def _u0(d, seed):
    rng = np.random.default_rng(seed)
    q, _ = np.linalg.qr(rng.standard_normal((d, d)))
    return q.astype(np.float32)


@pytest.mark.parametrize("N,d,K", [(256, 16, 4), (1000, 64, 4), (20000, 64, 4), (4099, 64, 8),
                                   (777, 32, 2), (3000, 128, 16), (50, 64, 1), (2048, 128, 4),
                                   (1, 16, 2), (640, 64, 64)])
def test_step_matches_oracle(N, d, K):
    from drsa_audio_amd.xai.drsa.drsa import drsa_step
    A, C = drsa_inputs(N, d, 1000 + N)
    U0 = _u0(d, d + K)
    Ug, Cg, Ag = _gpu(U0, C, A)
    Un, f = drsa_step(Ag, Cg, Ug, K)
    torch.cuda.synchronize()
    f_ref, G, _, _ = drsa_ref.closed_form(A, C, U0, K)
    assert abs(float(f) - f_ref) <= 1e-5 * abs(f_ref) + 1e-12
    Uref = drsa_ref.polar(U0.astype(np.float64) + G)
    Un = Un.cpu().numpy()
    assert np.abs(Un - Uref).max() < 2e-5
    assert np.abs(Un.T @ Un - np.eye(d)).max() < 2e-6


@pytest.mark.parametrize("tag", ["small", "c3w"])
def test_trajectory_vs_reference_fixture(fx, tag):
    from drsa_audio_amd.xai.drsa.drsa import drsa_run
    N, d, K, seed, steps = fx[f"{tag}_meta"]
    A, C = drsa_inputs(N, d, seed)
    Ag, Cg, Ug = _gpu(A, C, fx[f"{tag}_U0"])
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        U, traj = drsa_run(Ag, Cg, Ug, int(K), int(steps))
    torch.cuda.synchronize()
    traj = traj.cpu().numpy().astype(np.float64)
    ref = fx[f"{tag}_traj"]
    assert traj.shape == ref.shape
    assert np.max(np.abs(traj - ref) / np.abs(ref)) < 1e-4
    assert np.abs(U.cpu().numpy() - fx[f"{tag}_Ufinal"]).max() < 1e-4


def test_graph_and_eager_runs_identical():
    from drsa_audio_amd.xai.drsa.drsa import drsa_run
    A, C = drsa_inputs(5000, 64, 77)
    Ag, Cg, Ug = _gpu(A, C, _u0(64, 3))
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        U1, t1 = drsa_run(Ag, Cg, Ug, 4, 7, use_graph=True)
        U2, t2 = drsa_run(Ag, Cg, Ug, 4, 7, use_graph=False)
    torch.cuda.synchronize()
    assert torch.equal(U1, U2) and torch.equal(t1, t2)


@pytest.mark.parametrize("N,d,K", [(20000, 64, 4), (9001, 64, 8), (3000, 48, 4), (777, 64, 16), (20000, 128, 16),
                                   (3000, 100, 4), (2048, 128, 8), (4000, 128, 2), (1500, 72, 9), (777, 66, 2)])
def test_fused_run_equals_partial_finish_loop_bitwise(N, d, K):
    """drsa_run at DP = 64 takes the fused step (drsa_fused_step_kernel: the previous step's finish
    redone in every workgroup, then the partial on the new U from LDS), at DP = 128 the cooperative
    finish (drsa_finish_coop_kernel: the polar over 8 workgroups of 16 columns, including concept
    width 64 and heavily padded d = 66 / 72).  Its trajectory and U must equal, bit for bit, the
    explicit loop of the partial and the one-workgroup finish entry points."""
    from drsa_audio_amd import _capi
    from drsa_audio_amd.xai.drsa.drsa import DrsaWorkspace, drsa_run
    steps = 6
    A, C = drsa_inputs(N, d, 31)
    Ag, Cg, Ug = _gpu(A, C, _u0(d, 8))
    side = torch.cuda.Stream()   # a non-default stream: drsa_run replays its hipGraph
    with torch.cuda.stream(side):
        U_run, traj = drsa_run(Ag, Cg, Ug, K, steps)
    torch.cuda.synchronize()
    ws = DrsaWorkspace(N, d, K, DEV)
    st = _capi.stream_ptr()
    gs = ws.gs
    f = torch.empty(steps + 1, device=DEV)
    U = Ug.clone()
    for t in range(steps + 1):
        _capi.call("drsa_amd_drsa_partial", Ag.data_ptr(), Cg.data_ptr(), N, d, K, U.data_ptr(), gs.data_ptr(),
                   ws.ptr, ws.nbytes, st)
        U_new = torch.empty_like(U)
        _capi.call("drsa_amd_drsa_finish", gs.data_ptr(), N, d, K, U.data_ptr(), U_new.data_ptr(),
                   f[t:].data_ptr(), 1 if t == steps else 0, None, st)
        if t < steps:
            U = U_new
    torch.cuda.synchronize()
    assert torch.equal(torch.as_tensor(traj).to(f), f), (traj, f)
    assert torch.equal(U_run, U)


def test_coop_finish_timeout_is_loud_and_recoverable():
    """VERDICT r05 item 2 / ADVICE r05: the cooperative DP = 128 finish must never fail silently.
    With the spin budget forced to 0 (drsa_amd_debug_coop_spin_budget) some workgroup gives up at its
    first poll that finds a partner missing: drsa_run must raise DrsaAmdError (DRSA_ETIMEOUT), the
    workspace's status word must read 1, U must be NaN, and the run's later finishes must skip
    straight to NaN (no 100 ms spins: the 40-step run ends in well under a second).  With the budget
    restored the next run on the same workspace succeeds and equals a fresh workspace's run bit
    for bit (coop_reset clears the ticket and the status per run)."""
    import time
    from drsa_audio_amd import _capi
    from drsa_audio_amd.xai.drsa.drsa import DrsaWorkspace, drsa_run
    N, d, K, steps = 4096, 128, 16, 40
    A, C = drsa_inputs(N, d, 5)
    Ag, Cg, Ug = _gpu(A, C, _u0(d, 2))
    ws = DrsaWorkspace(N, d, K, DEV)
    side = torch.cuda.Stream()
    _capi.call("drsa_amd_debug_coop_spin_budget", 0)
    try:
        t0 = time.time()
        with torch.cuda.stream(side):
            with pytest.raises(_capi.DrsaAmdError, match="timed out"):
                drsa_run(Ag, Cg, Ug, K, steps, ws=ws)
        torch.cuda.synchronize()
        assert time.time() - t0 < 5.0
        assert ws.coop_status() == 1
    finally:
        _capi.call("drsa_amd_debug_coop_spin_budget", -1)
    with torch.cuda.stream(side):
        U1, t1 = drsa_run(Ag, Cg, Ug, K, steps, ws=ws)
        U2, t2 = drsa_run(Ag, Cg, Ug, K, steps)
    torch.cuda.synchronize()
    assert ws.coop_status() == 0
    assert torch.isfinite(U1).all() and torch.isfinite(t1).all()
    assert torch.equal(U1, U2) and torch.equal(t1, t2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_joint_run_captured_in_caller_graph_equals_eager(dtype):
    """drsa_amd_drsa_run_multi inside a caller's stream capture (bench.py's steady-state timing,
    VERDICT r05 item 2): it records its forked per-problem chains into the caller's graph; two
    replays of that graph give the eager joint run's trajectories and U bit for bit (d = 128 takes
    the cooperative finish, whose status word stays 0)."""
    from drsa_audio_amd.xai.drsa.drsa import drsa_run_joint
    N, d, K, steps = 3000, 128, 16, 7
    probs = []
    for seed in (1, 2):
        A, C = drsa_inputs(N, d, seed)
        Ag, Cg, Ug = _gpu(A, C, _u0(d, seed))
        probs.append((Ag.to(dtype), Cg.to(dtype), Ug, K))
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        ref = drsa_run_joint(probs, steps)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        out = drsa_run_joint(probs, steps)
    for _ in range(2):
        with torch.cuda.stream(side):
            g.replay()
        torch.cuda.synchronize()
        for (U, t), (Ur, tr) in zip(out, ref):
            assert torch.equal(t, tr) and torch.equal(U, Ur)


def test_sharded_fused_step_equals_two_call_form_bitwise():
    """sharded_run's fused path (drsa_amd_drsa_fused_step: finish + the next partial in one
    launch, caller-owned buffers) equals the partial / finish two-call form bit for bit."""
    from drsa_audio_amd.xai.drsa.distributed import HipBackend, sharded_run

    class TwoCall(HipBackend):
        def fused_supported(self):
            return False

    for N, d, K in ((9001, 64, 8), (3000, 48, 4)):
        A, C = drsa_inputs(N, d, 41)
        Ag, Cg, Ug = _gpu(A, C, _u0(d, 12))
        assert HipBackend(Ag, Cg, d, K).fused_supported()
        U1, t1 = sharded_run(Ag, Cg, Ug, K, 7)
        U2, t2 = sharded_run(Ag, Cg, Ug, K, 7, backend=TwoCall(Ag, Cg, d, K))
        assert np.array_equal(t1, t2) and torch.equal(U1, U2)


def test_sharded_joint_preallocated_equals_generic_loop_bitwise():
    """sharded_run_joint with HIP backends (partials written into one packed all-reduce buffer,
    preallocated U / trajectory) equals the generic backend loop bit for bit (C5 shapes)."""
    from drsa_audio_amd.xai.drsa.distributed import HipBackend, sharded_run_joint

    class Wrap:   # not a HipBackend: takes the generic loop
        def __init__(self, b):
            self.b = b

        def slab_size(self):
            return self.b.slab_size()

        def partial(self, U):
            return self.b.partial(U)

        def finish(self, gs, N, U):
            return self.b.finish(gs, N, U)

        def objective(self, gs, N, U):
            return self.b.objective(gs, N, U)

    probs = []
    for seed, (N, d, K) in enumerate(((3000, 128, 16), (2500, 64, 8))):
        A, C = drsa_inputs(N, d, 60 + seed)
        Ag, Cg, Ug = _gpu(A, C, _u0(d, 20 + seed))
        probs.append((Ag, Cg, Ug, K))
    fast = sharded_run_joint(probs, 5)
    slow = sharded_run_joint(probs, 5, backends=[Wrap(HipBackend(A, C, U.size(0), K)) for A, C, U, K in probs])
    for (U1, t1), (U2, t2) in zip(fast, slow):
        assert np.array_equal(t1, t2) and torch.equal(U1, U2)


def test_deterministic_bitwise():
    from drsa_audio_amd.xai.drsa.drsa import drsa_step
    A, C = drsa_inputs(30000, 64, 5)
    Ag, Cg, Ug = _gpu(A, C, _u0(64, 9))
    a = drsa_step(Ag, Cg, Ug, 4)
    b = drsa_step(Ag, Cg, Ug, 4)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


def test_sharded_partials_sum_to_full():
    """The multi-GPU step: per-shard partial, sum (all-reduce), finish with global N."""
    from drsa_audio_amd import _capi
    from drsa_audio_amd.xai.drsa.drsa import DrsaWorkspace, drsa_step
    N, d, K = 8000, 64, 8
    A, C = drsa_inputs(N, d, 21)
    Ag, Cg, Ug = _gpu(A, C, _u0(64, 4))
    parts = []
    st = _capi.stream_ptr()
    for sl in (slice(0, 2500), slice(2500, 6001), slice(6001, N)):
        a, c = Ag[sl].contiguous(), Cg[sl].contiguous()
        ws = DrsaWorkspace(a.size(0), d, K, DEV)
        gs = torch.empty(d * d + K, device=DEV)
        _capi.call("drsa_amd_drsa_partial", a.data_ptr(), c.data_ptr(), a.size(0), d, K, Ug.data_ptr(),
                   gs.data_ptr(), ws.ptr, ws.nbytes, st)
        parts.append(gs)
    gsum = parts[0] + parts[1] + parts[2]
    U_new = torch.empty_like(Ug)
    f = torch.empty(1, device=DEV)
    _capi.call("drsa_amd_drsa_finish", gsum.data_ptr(), N, d, K, Ug.data_ptr(), U_new.data_ptr(),
               f.data_ptr(), 0, None, st)
    U_full, f_full = drsa_step(Ag, Cg, Ug, K)
    assert abs(float(f) - float(f_full)) <= 1e-6 * abs(float(f_full))
    assert (U_new - U_full).abs().max().item() < 1e-5


def test_orthogonalize_api():
    from drsa_audio_amd.xai.drsa.drsa import orthogonalize
    rng = np.random.default_rng(3)
    for d in (16, 32, 64, 128):
        V = (np.eye(d) + 0.3 * rng.standard_normal((d, d))).astype(np.float32)
        out = orthogonalize(_gpu(V)[0]).cpu().numpy()
        assert np.abs(out - drsa_ref.polar(V)).max() < 5e-5
        assert np.abs(out.T @ out - np.eye(d)).max() < 5e-6


def test_objective_api_and_optimizer_files(tmp_path, fx):
    from drsa_audio_amd.xai.drsa.drsa import SubspaceOptimizer, objective_fn
    N, d, K, seed, steps = fx["small_meta"]
    A, C = drsa_inputs(N, d, seed)
    Ag, Cg, Ug = _gpu(A, C, fx["small_U0"])
    f = SubspaceOptimizer.obj_val(Ag, Cg, Ug, objective_fn, int(K), int(d // K))
    assert abs(float(f) - float(fx["small_f0"])) <= 1e-5 * float(fx["small_f0"])
    opt = SubspaceOptimizer(Ug, Ag, Cg, str(tmp_path), num_concepts=int(K), device="cuda")
    opt.run(steps=int(steps))
    import pandas as pd, pickle
    df = pd.read_csv(tmp_path / "train_stats.csv")
    assert list(df.columns) == ["Unnamed: 0", "loss"] and len(df) == steps + 1
    assert np.max(np.abs(df["loss"].values - fx["small_traj"]) / fx["small_traj"]) < 1e-4
    with open(tmp_path / "projection_matrix.pkl", "rb") as fh:   # file written by this test
        U = pickle.load(fh)
    assert U.dtype == np.float32 and U.shape == (d, d)


def _sharded_worker(rank, world, port, A, C, U0, K, steps, q):
    import os, sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from drsa_audio_amd.xai.drsa.distributed import shard_rows, sharded_run
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    sl = shard_rows(A.shape[0], world, rank)
    U, traj = sharded_run(torch.from_numpy(A[sl]).to(dev), torch.from_numpy(C[sl]).to(dev),
                          torch.from_numpy(U0).to(dev), K, steps)
    q.put((rank, U.cpu().numpy(), traj))
    dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_run_two_ranks_gloo_matches_single():
    """Two ranks on cuda:0 (gloo carries the [d*d+K] all-reduce): identical U on both ranks and
    the same trajectory as the single-process HIP run up to the partial-sum order."""
    import socket
    import torch.multiprocessing as mp
    from gen_fixtures import drsa_inputs
    from drsa_audio_amd.xai.drsa.drsa import DrsaWorkspace, drsa_run
    A, C = drsa_inputs(5001, 64, 11)
    U0 = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "u64_seed42.npy"))
    K, steps = 4, 20
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_sharded_worker, args=(r, 2, port, A, C, U0, K, steps, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: (u, t) for r, u, t in (q.get(timeout=300) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.array_equal(res[0][0], res[1][0]) and np.array_equal(res[0][1], res[1][1])
    dev = torch.device("cuda", 0)
    ws = DrsaWorkspace(A.shape[0], 64, K, dev)
    U1, traj1 = drsa_run(torch.from_numpy(A).to(dev), torch.from_numpy(C).to(dev), torch.from_numpy(U0).to(dev),
                         K, steps, ws)
    traj1 = traj1.cpu().numpy()
    assert np.max(np.abs(res[0][1] - traj1) / np.abs(traj1)) < 1e-5
    assert np.abs(res[0][0] - U1.cpu().numpy()).max() < 1e-4


def test_joint_run_equals_separate_runs_bitwise():
    """drsa_amd_drsa_run_multi (C5: two d=128 K=16 problems in one graph) gives exactly what two
    separate drsa_run calls give."""
    from drsa_audio_amd.xai.drsa.drsa import drsa_run, drsa_run_joint
    probs = []
    for N, seed in ((3000, 1), (2048, 2)):
        A, C = drsa_inputs(N, 128, seed)
        probs.append((*_gpu(A, C, _u0(128, seed)), 16))
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        joint = drsa_run_joint(probs, 7)
        sep = [drsa_run(A, C, U0, K, 7) for A, C, U0, K in probs]
    torch.cuda.synchronize()
    for (Uj, tj), (Us, ts) in zip(joint, sep):
        assert torch.equal(Uj, Us) and torch.equal(tj, ts)
    # and against the oracle's trajectory
    A, C, U0, K = probs[0]
    Ur, ref = drsa_ref.run(A.cpu(), C.cpu(), U0.cpu(), K, 7)
    np.testing.assert_allclose(joint[0][1].cpu().numpy(), np.array(ref), rtol=1e-4)


@pytest.mark.parametrize("N,d,K", [(3000, 64, 4), (2048, 128, 16), (777, 32, 2), (20000, 64, 8)])
@pytest.mark.parametrize("dt", ["bf16", "f16"])
def test_bf16_partial_matches_bf16_closed_form(N, d, K, dt):
    """16-bit paths (C5: bf16 / fp16 MFMA projection): the kernel against the float64 closed form
    ON THE SAME 16-bit inputs (tight: 2e-5 relative) — checks the MFMA operand layout and the
    widening, not the rounding."""
    from drsa_audio_amd.xai.drsa.drsa import DrsaWorkspace
    from drsa_audio_amd import _capi
    rnd = drsa_ref.bf16_round if dt == "bf16" else drsa_ref.f16_round
    tdt = torch.bfloat16 if dt == "bf16" else torch.float16
    A, C = drsa_inputs(N, d, 7000 + N)
    Ab, Cb = rnd(A), rnd(C)
    U0 = _u0(d, d + K)
    At = torch.from_numpy(Ab).to(DEV).to(tdt)
    Ct = torch.from_numpy(Cb).to(DEV).to(tdt)
    Ut = torch.from_numpy(U0).to(DEV)
    ws = DrsaWorkspace(N, d, K, DEV)
    gs = torch.empty(d * d + K, device=DEV)
    _capi.call(f"drsa_amd_drsa_partial_{dt}", At.data_ptr(), Ct.data_ptr(), N, d, K, Ut.data_ptr(), gs.data_ptr(),
               ws.ptr, ws.nbytes, _capi.stream_ptr(DEV))
    torch.cuda.synchronize()
    f_ref, G_ref = drsa_ref.closed_form_bf16(Ab, Cb, U0, K, rounder=rnd)
    Ud = rnd(U0).astype(np.float64)
    XA, XC = Ab.astype(np.float64) @ Ud, Cb.astype(np.float64) @ Ud
    r = np.maximum((XA * XC).reshape(N, K, d // K).sum(-1), 0)
    S_ref = (r * r).sum(0)
    S = gs[d * d:].cpu().numpy().astype(np.float64)
    np.testing.assert_allclose(S, S_ref, rtol=2e-5, atol=1e-6 * S_ref.max())
    # unscaled gradient = A^T (R (.) XC) + C^T (R (.) XA)
    R = np.repeat(r, d // K, axis=1)
    Gt = Ab.astype(np.float64).T @ (R * XC) + Cb.astype(np.float64).T @ (R * XA)
    Gk = gs[:d * d].cpu().numpy().reshape(d, d).astype(np.float64)
    assert np.abs(Gk - Gt).max() <= 2e-5 * np.abs(Gt).max()


@pytest.mark.parametrize("tdt", [torch.bfloat16, torch.float16])
def test_bf16_joint_run_objective_within_loosened_tolerance(tdt):
    """C5 bf16 / fp16 vs the fp32 path on the same (unrounded) data: the DRSA objective
    trajectory stays within 1e-2 relative (loosened tolerance for a path the reference does not
    have)."""
    from drsa_audio_amd.xai.drsa.drsa import drsa_run, drsa_run_joint
    probs32, probs16 = [], []
    for N, seed in ((4000, 26), (3000, 33)):
        A, C = drsa_inputs(N, 128, seed)
        U0 = _u0(128, seed)
        A32, C32, U = _gpu(A, C, U0)
        probs32.append((A32, C32, U, 16))
        probs16.append((A32.to(tdt), C32.to(tdt), U, 16))
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        j16 = drsa_run_joint(probs16, 20)
        j32 = drsa_run_joint(probs32, 20)
        one16 = drsa_run(*probs16[0], 20)
    torch.cuda.synchronize()
    for (U16, t16), (U32, t32) in zip(j16, j32):
        t16, t32 = t16.cpu().numpy(), t32.cpu().numpy()
        assert np.all(np.abs(t16 - t32) <= 1e-2 * np.abs(t32)), (t16, t32)
        assert t16[-1] > t16[0]                       # still ascending
        Un = U16.cpu().double().numpy()
        assert np.abs(Un.T @ Un - np.eye(128)).max() < 1e-5
    assert torch.equal(one16[1], j16[0][1])           # single-problem bf16 route = joint route


def _rccl_graph_worker(port, A, C, U0, K, steps, q):
    """One rank over RCCL (nccl backend, world size 1): the sharded loops with the step graph
    (all-reduce captured) and eagerly, C4-shape fused and C5-shape joint."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    from drsa_audio_amd.xai.drsa import distributed as D
    out = {}
    Ag, Cg, Ug = (torch.from_numpy(v).to(dev) for v in (A, C, U0))
    g = torch.Generator().manual_seed(3)
    U5 = [torch.linalg.qr(torch.randn(128, 128, generator=g, dtype=torch.float64))[0].float().to(dev) for _ in range(2)]
    probs = []
    for p_ in range(2):
        A5, C5 = drsa_inputs(3000, 128, 40 + p_)
        probs.append((torch.from_numpy(A5).to(dev), torch.from_numpy(C5).to(dev), U5[p_], 16))
    for mode in ("1", "0"):
        os.environ["DRSA_AMD_SHARDED_GRAPH"] = mode
        U, tr = D.sharded_run(Ag, Cg, Ug, K, steps)
        joint = D.sharded_run_joint(probs, 7)
        out[mode] = (U.cpu().numpy(), tr, [(u.cpu().numpy(), t) for u, t in joint])
        if mode == "1":
            out["stats"] = dict(D.STATS)
    dist.destroy_process_group()
    q.put(out)


@pytest.mark.gpu
def test_sharded_step_graph_over_rccl_equals_eager():
    """The captured sharded step (RCCL all-reduce + fused step in one graph, replayed; odd step
    counts finish eagerly) gives exactly the eager loop's U and trajectory, fused and joint."""
    import socket
    import torch.multiprocessing as mp
    A, C = drsa_inputs(20000, 64, 12)
    U0 = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "u64_seed42.npy"))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_graph_worker, args=(port, A, C, U0, 8, 11, q))
    p.start()
    out = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    g, e = out["1"], out["0"]
    assert out["stats"]["graph_replays"] == 5 + 3 and out["stats"]["capture_failures"] == 0, out["stats"]
    assert np.array_equal(g[0], e[0]) and np.array_equal(g[1], e[1])
    assert len(g[1]) == 12 and np.all(np.isfinite(g[1]))
    for (ug, tg), (ue, te) in zip(g[2], e[2]):
        assert np.array_equal(ug, ue) and np.array_equal(tg, te)
