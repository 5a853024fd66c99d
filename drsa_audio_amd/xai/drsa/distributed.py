"""Row-sharded DRSA optimisation across ranks (one process per GPU).

Each rank holds a shard of the activation/context rows.  One step:

    gs_local = [A_r^T (R (.) C_r U) + C_r^T (R (.) A_r U)  |  S_k,r]     (drsa_amd_drsa_partial)
    gs       = all_reduce(gs_local, SUM)                                  (RCCL over xGMI: slab fp32)
    f, U'    = finish(gs, N_total)                                         (drsa_amd_drsa_finish)

The all-reduce payload is 16.4 KB at d=64 (64.1 KB at d=128): latency-bound, one collective
per step.  Every rank receives identical reduced bytes and runs the identical deterministic
polar step, so U stays replicated without a broadcast.  The step math is the reference's
(``drsa.py:84-106``); sharding is exact up to the fp32 summation order of the partials.

The per-step kernels are pluggable (``backend``) so the orchestration is tested on CPU with
gloo (tests/test_dist_cpu.py) using the oracle's closed form; the product backend is HIP.  Over
RCCL the step loop is captured once in a graph -- the all-reduce and the step kernels of two steps
-- and replayed (the trajectory slot advances through a device counter), so no Python or launch
work sits between steps; DRSA_AMD_SHARDED_GRAPH=0 runs it eagerly (same kernels, same bits).
"""
from __future__ import annotations

import os
from typing import Callable, List, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from ... import _capi


class HipBackend:
    """libdrsa_amd kernels on the rank's GPU."""

    def __init__(self, A: torch.Tensor, C: torch.Tensor, d: int, K: int):
        from .drsa import DrsaWorkspace, slab_floats
        self.A, self.C, self.d, self.K = A, C, d, K
        self.ws = DrsaWorkspace(max(A.size(0), 1), d, K, A.device)
        self.gs = torch.empty(slab_floats(d, K), device=A.device, dtype=torch.float32)
        self.f = torch.empty(1, device=A.device, dtype=torch.float32)

    def slab_size(self) -> int:
        return self.gs.numel()

    def partial(self, U: torch.Tensor) -> torch.Tensor:
        _capi.call("drsa_amd_drsa_partial", self.A.data_ptr(), self.C.data_ptr(), self.A.size(0), self.d, self.K,
                   U.data_ptr(), self.gs.data_ptr(), self.ws.ptr, self.ws.nbytes, _capi.stream_ptr(U.device))
        return self.gs

    def finish(self, gs: torch.Tensor, N_total: int, U: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        U_new = torch.empty_like(U)
        _capi.call("drsa_amd_drsa_finish", gs.data_ptr(), int(N_total), self.d, self.K, U.data_ptr(),
                   U_new.data_ptr(), self.f.data_ptr(), 0, None, _capi.stream_ptr(U.device))
        return U_new, self.f.clone()

    def finish_into(self, gs: torch.Tensor, N_total: int, U: torch.Tensor, U_out: torch.Tensor,
                    f_out: torch.Tensor) -> None:
        """finish() into caller-owned buffers (f(U) -> f_out[0])."""
        _capi.call("drsa_amd_drsa_finish", gs.data_ptr(), int(N_total), self.d, self.K, U.data_ptr(),
                   U_out.data_ptr(), f_out.data_ptr(), 0, None, _capi.stream_ptr(U.device))

    def fused_supported(self) -> bool:
        return bool(_capi.load().drsa_amd_drsa_fused_supported(self.d, self.K))

    def fused(self, gs: torch.Tensor, N_total: int, U: torch.Tensor, U_out: torch.Tensor, f_out: torch.Tensor,
              gs_out: torch.Tensor) -> None:
        """finish(gs) -> U_out, f(U) -> f_out[0], then partial at U_out -> gs_out, in one launch
        fewer (drsa_amd_drsa_fused_step); everything written into caller-owned buffers."""
        _capi.call("drsa_amd_drsa_fused_step", self.A.data_ptr(), self.C.data_ptr(), self.A.size(0), self.d, self.K,
                   gs.data_ptr(), int(N_total), U.data_ptr(), U_out.data_ptr(), f_out.data_ptr(), gs_out.data_ptr(),
                   self.ws.ptr, self.ws.nbytes, _capi.stream_ptr(U.device))

    def fused_counted(self, gs: torch.Tensor, N_total: int, U: torch.Tensor, U_out: torch.Tensor,
                      f_traj: torch.Tensor, counter: torch.Tensor, gs_out: torch.Tensor) -> None:
        """fused() with f(U) -> f_traj[*counter], counter += 1 on the device (graph replays)."""
        _capi.call("drsa_amd_drsa_fused_step_counted", self.A.data_ptr(), self.C.data_ptr(), self.A.size(0), self.d,
                   self.K, gs.data_ptr(), int(N_total), U.data_ptr(), U_out.data_ptr(), f_traj.data_ptr(),
                   counter.data_ptr(), gs_out.data_ptr(), self.ws.ptr, self.ws.nbytes, _capi.stream_ptr(U.device))

    def finish_counted(self, gs: torch.Tensor, N_total: int, U: torch.Tensor, U_out: torch.Tensor,
                       f_traj: torch.Tensor, counter: torch.Tensor) -> None:
        _capi.call("drsa_amd_drsa_finish_counted", gs.data_ptr(), int(N_total), self.d, self.K, U.data_ptr(),
                   U_out.data_ptr(), f_traj.data_ptr(), counter.data_ptr(), _capi.stream_ptr(U.device))

    def objective(self, gs: torch.Tensor, N_total: int, U: torch.Tensor) -> torch.Tensor:
        _capi.call("drsa_amd_drsa_finish", gs.data_ptr(), int(N_total), self.d, self.K, U.data_ptr(), None,
                   self.f.data_ptr(), 1, None, _capi.stream_ptr(U.device))
        return self.f.clone()


# graph replays issued by the sharded loops in this process (tests check the graph path ran)
STATS = {"graph_replays": 0, "capture_failures": 0}


def _graph_ok(group, backends) -> bool:
    """Capture the step loop (kernels + the RCCL all-reduce) in a graph: RCCL process group, HIP
    backends and DRSA_AMD_SHARDED_GRAPH.  Default ("auto"): only at world size 1 -- a captured
    multi-rank RCCL all-reduce has not yet been checked against the eager loop on two GPUs;
    DRSA_AMD_SHARDED_GRAPH=1 enables it at any world size, 0 disables it."""
    mode = os.environ.get("DRSA_AMD_SHARDED_GRAPH", "auto")
    if mode == "0" or not dist.is_initialized():
        return False
    if not all(isinstance(b, HipBackend) for b in backends):
        return False
    try:
        if dist.get_backend(group) != "nccl":
            return False
    except Exception:
        return False
    return mode == "1" or dist.get_world_size(group) == 1


def _capture(body, group=None) -> Optional["torch.cuda.CUDAGraph"]:
    """One captured replay of ``body`` (two steps: U ping-pongs back to its buffer), or None when
    the capture is refused (then the loop runs eagerly, same kernels and the same bits).  The
    ranks agree first (MIN of a success flag over the group): either every rank replays the graph
    or every rank runs eagerly."""
    g = torch.cuda.CUDAGraph()
    ok = 1
    try:
        with torch.cuda.graph(g):
            body()
    except Exception:
        torch.cuda.synchronize()
        STATS["capture_failures"] += 1
        ok = 0
    if dist.is_initialized():
        flag = torch.tensor([ok], dtype=torch.int32, device=torch.device("cuda", torch.cuda.current_device()))
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
        ok = int(flag.item())
    return g if ok else None


def sharded_run(A_local: torch.Tensor, C_local: torch.Tensor, U0: torch.Tensor, K: int, steps: int,
                group=None, backend=None) -> Tuple[torch.Tensor, np.ndarray]:
    """SubspaceOptimizer.run over row shards.  Returns (U_steps, trajectory [steps+1]) on every rank."""
    d = U0.size(0)
    backend = backend or HipBackend(A_local.contiguous(), C_local.contiguous(), d, K)
    n = torch.tensor([A_local.size(0)], dtype=torch.int64, device=U0.device)
    if dist.is_initialized():
        dist.all_reduce(n, op=dist.ReduceOp.SUM, group=group)
    N_total = int(n.item())
    if getattr(backend, "fused_supported", lambda: False)() and A_local.size(0) > 0:
        # fused steps: all-reduce(partials at U_t) -> [finish t + partial at U_t+1] -> ...; U ping-pongs
        # between two buffers and f lands in its trajectory slot (no per-step allocation)
        Ub = [U0.detach().clone().contiguous(), torch.empty_like(U0)]
        traj_t = torch.empty(steps + 1, device=U0.device, dtype=torch.float32)
        counter = torch.zeros(1, device=U0.device, dtype=torch.int32)   # f(U_t) -> traj_t[counter++]
        gs = backend.partial(Ub[0])

        def step(t):
            if dist.is_initialized():
                dist.all_reduce(gs, op=dist.ReduceOp.SUM, group=group)
            backend.fused_counted(gs, N_total, Ub[t % 2], Ub[(t + 1) % 2], traj_t, counter, gs)

        t0 = 0
        if steps >= 4 and _graph_ok(group, [backend]):
            # the whole step (all-reduce + fused launch) replayed from one graph, two steps per replay
            graph = _capture(lambda: (step(0), step(1)), group)
            if graph is not None:
                for _ in range(steps // 2):
                    graph.replay()
                STATS["graph_replays"] += steps // 2
                t0 = 2 * (steps // 2)
        for t in range(t0, steps):
            step(t)
        if dist.is_initialized():
            dist.all_reduce(gs, op=dist.ReduceOp.SUM, group=group)
        traj_t[steps:] = backend.objective(gs, N_total, Ub[steps % 2])
        return Ub[steps % 2], traj_t.cpu().numpy()
    U = U0.detach().clone().contiguous()
    traj: List[torch.Tensor] = []
    for _ in range(steps):
        gs = backend.partial(U)
        if dist.is_initialized():
            dist.all_reduce(gs, op=dist.ReduceOp.SUM, group=group)
        U, f = backend.finish(gs, N_total, U)
        traj.append(f)
    gs = backend.partial(U)
    if dist.is_initialized():
        dist.all_reduce(gs, op=dist.ReduceOp.SUM, group=group)
    traj.append(backend.objective(gs, N_total, U))
    return U, torch.cat([t.reshape(1) for t in traj]).cpu().numpy()


def sharded_run_joint(problems, steps: int, group=None, backends=None):
    """Several DRSA problems (C5: layers j=26 and j=33 of one model, K=16 each) row-sharded over
    the process group and advanced together with ONE all-reduce per step: the P partials
    [d_p*d_p + K_p] are packed into one buffer (64.1 KB per d=128 problem), reduced, and each
    problem finishes from its slice.  ``problems``: list of (A_local, C_local, U0, K).
    Returns [(U_S, trajectory [S+1])] on every rank."""
    P = len(problems)
    if backends is None:
        backends = [HipBackend(A.contiguous(), C.contiguous(), U0.size(0), K) for A, C, U0, K in problems]
    dev = problems[0][2].device
    n = torch.tensor([A.size(0) for A, _, _, _ in problems], dtype=torch.int64, device=dev)
    if dist.is_initialized():
        dist.all_reduce(n, op=dist.ReduceOp.SUM, group=group)
    N_tot = [int(v) for v in n.tolist()]
    sizes = [b.slab_size() for b in backends]
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(int)
    if all(isinstance(b, HipBackend) for b in backends):
        # the partials land straight in their slices of ONE packed all-reduce buffer, U ping-pongs
        # between preallocated buffers and f goes to its trajectory slot: no per-step allocation
        packed = torch.empty(int(offs[-1]), device=dev, dtype=torch.float32)
        for p, b in enumerate(backends):
            b.gs = packed[offs[p]:offs[p + 1]]
        Ub = [[U0.detach().clone().contiguous(), torch.empty_like(U0)] for _, _, U0, _ in problems]
        tr = [torch.empty(steps + 1, device=dev, dtype=torch.float32) for _ in range(P)]

        def reduce_all(Ucur):
            for p in range(P):
                backends[p].partial(Ucur[p])
            if dist.is_initialized():
                dist.all_reduce(packed, op=dist.ReduceOp.SUM, group=group)

        counters = [torch.zeros(1, device=dev, dtype=torch.int32) for _ in range(P)]
        # the P finishes (single-workgroup polar each) run concurrently: problems 1.. on side streams
        side = [torch.cuda.Stream(device=dev) for _ in range(P - 1)]

        def step(t):
            reduce_all([Ub[p][t % 2] for p in range(P)])
            cur = torch.cuda.current_stream(dev)
            ev = torch.cuda.Event()
            ev.record(cur)
            for p in range(P):
                st = cur if p == 0 else side[p - 1]
                if p:
                    st.wait_event(ev)
                with torch.cuda.stream(st):
                    backends[p].finish_counted(backends[p].gs, N_tot[p], Ub[p][t % 2], Ub[p][(t + 1) % 2], tr[p],
                                               counters[p])
            for st in side:
                cur.wait_stream(st)

        t0 = 0
        if steps >= 4 and _graph_ok(group, backends):
            graph = _capture(lambda: (step(0), step(1)), group)
            if graph is not None:
                for _ in range(steps // 2):
                    graph.replay()
                STATS["graph_replays"] += steps // 2
                t0 = 2 * (steps // 2)
        for t in range(t0, steps):
            step(t)
        reduce_all([Ub[p][steps % 2] for p in range(P)])
        out = []
        for p in range(P):
            tr[p][steps:] = backends[p].objective(backends[p].gs, N_tot[p], Ub[p][steps % 2])
            out.append((Ub[p][steps % 2], tr[p].cpu().numpy()))
        return out
    Us = [U0.detach().clone().contiguous() for _, _, U0, _ in problems]
    trajs: List[List[torch.Tensor]] = [[] for _ in range(P)]

    def reduced():
        parts = [backends[p].partial(Us[p]) for p in range(P)]
        buf = torch.cat([t.reshape(-1) for t in parts])
        if dist.is_initialized():
            dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
        return [buf[offs[p]:offs[p + 1]].contiguous() for p in range(P)]

    for _ in range(steps):
        gss = reduced()
        for p in range(P):
            Us[p], f = backends[p].finish(gss[p], N_tot[p], Us[p])
            trajs[p].append(f)
    gss = reduced()
    out = []
    for p in range(P):
        trajs[p].append(backends[p].objective(gss[p], N_tot[p], Us[p]))
        out.append((Us[p], torch.cat([t.reshape(1) for t in trajs[p]]).cpu().numpy()))
    return out


def shard_rows(N: int, world: int, rank: int) -> slice:
    """Contiguous, balanced row range of ``rank``."""
    base, rem = divmod(N, world)
    start = rank * base + min(rank, rem)
    return slice(start, start + base + (1 if rank < rem else 0))


def main_sharded(activation_vecs: torch.Tensor, context_vecs: torch.Tensor, model_root: str,
                 num_concepts: int = 4, steps: int = 2000, runs: int = 3, seed: int = 42,
                 local_rows: bool = False, group=None) -> Optional[List[str]]:
    """drsa.main semantics (drsa.py:241-301) with the rows split over the process group; rank 0
    writes ``run{r}/projection_matrix.pkl`` and ``run{r}/train_stats.csv``.

    ``local_rows=False``: every rank passes the whole (A, C) and keeps its ``shard_rows`` range.
    ``local_rows=True``: every rank passes only its own rows, e.g. from
    ``preprocessing.drsa_training_data(..., group=...)`` (no rank ever holds the full set)."""
    import pickle
    from .drsa import initial_projections
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    dev = torch.device("cuda", torch.cuda.current_device())
    sl = slice(None) if local_rows else shard_rows(activation_vecs.size(0), world, rank)
    A = activation_vecs[sl].to(dev, torch.float32).contiguous()
    C = context_vecs[sl].to(dev, torch.float32).contiguous()
    d = A.size(1)
    paths = []
    for r, U in enumerate(initial_projections(d, runs, seed), start=1):
        Uf, traj = sharded_run(A, C, torch.tensor(U, dtype=torch.float32, device=dev), num_concepts, steps,
                               group=group)
        if rank == 0:
            path = os.path.join(model_root, f"run{r}")
            os.makedirs(path, exist_ok=True)
            with open(os.path.join(path, "projection_matrix.pkl"), "wb") as fh:
                pickle.dump(Uf.cpu().numpy(), fh)
            import pandas as pd
            pd.DataFrame({"loss": [np.asarray(v, dtype=np.float32) for v in traj]}).to_csv(
                os.path.join(path, "train_stats.csv"))
            paths.append(path)
    return paths if rank == 0 else None
