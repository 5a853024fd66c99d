"""DRSA optimiser, drop-in for ``cxai.xai.drsa.drsa`` (reference ``cxai/xai/drsa/drsa.py``).

Every step runs on the GPU through ``libdrsa_amd.so``:

* objective + closed-form gradient in one fused pass over A, C (fp32 MFMA),
  deterministic slab reduction, then the objective scalars, the gradient scaling
  and the polar retraction (Newton–Schulz on MFMA) in one workgroup — no host
  round trip per step (the reference syncs twice per step, drsa.py:104,216);
* ``run`` launches the whole S-step loop natively (``drsa_amd_drsa_run``),
  replaying a captured hipGraph, and copies the trajectory back once.

Public names and argument meanings follow the reference:
``SubspaceOptimizer`` (drsa.py:15-168), ``generalized_fmean`` (171-182),
``project_grad`` (185-198), ``orthogonalize`` (201-221), ``objective_fn`` (224-238),
``main`` (241-301).  Outputs on disk are the same: ``run{r}/projection_matrix.pkl``
(pickled float32 numpy d×d) and ``run{r}/train_stats.csv`` (column ``loss``, S+1 rows).
"""
from __future__ import annotations

import os
import pickle
from typing import Callable, List, Optional

import numpy as np
import torch

from ... import _capi

__all__ = ["SubspaceOptimizer", "generalized_fmean", "project_grad", "orthogonalize",
           "objective_fn", "main", "DrsaWorkspace", "slab_floats", "drsa_run_batched"]


def _dev(device) -> torch.device:
    if device is None:
        return torch.device("cuda")
    device = torch.device(device) if isinstance(device, str) else device
    if device.type != "cuda":
        raise _capi.DrsaAmdError(f"drsa_audio_amd runs on the GPU only (got device={device})")
    return device


def slab_floats(d: int, K: int) -> int:
    """Floats of the [gradient | S] slab exchanged between drsa_partial and drsa_finish (the
    all-reduce payload of a sharded run): d*d + K for power-of-two shapes, padded coordinates
    otherwise (e.g. 128*128 + 4 for VGGish layer 19, d = 100, K = 4)."""
    n = _capi.lib().drsa_amd_drsa_slab_floats(int(d), int(K))
    if n == 0:
        raise _capi.DrsaAmdError(f"unsupported DRSA problem d={d} K={K} (d <= 128, K | d, d/K padded to a power "
                                 "of two <= 64 with K * padded width <= 128)")
    return int(n)


class DrsaWorkspace:
    """Device scratch for one (N, d, K) problem: partial slabs, reduced gradient, counters."""

    def __init__(self, N: int, d: int, K: int, device: torch.device):
        nbytes = _capi.lib().drsa_amd_drsa_workspace_bytes(int(N), int(d), int(K))
        if nbytes == 0:
            raise _capi.DrsaAmdError(f"unsupported DRSA problem N={N} d={d} K={K}")
        self.N, self.d, self.K = int(N), int(d), int(K)
        self.slab = int(slab_floats(d, K))
        self.buf = torch.empty(int(nbytes), dtype=torch.uint8, device=device)
        self.counter = torch.zeros(4, dtype=torch.int32, device=device)
        self.gs = torch.empty(self.slab, dtype=torch.float32, device=device)
        self.f = torch.empty(1, dtype=torch.float32, device=device)

    @property
    def ptr(self) -> int:
        return self.buf.data_ptr()

    @property
    def nbytes(self) -> int:
        return self.buf.numel()

    def coop_status(self) -> int:
        """1 if the cooperative finish of the last run on this workspace timed out (U, f NaN from
        that step on), else 0.  drsa_run raises on it by itself; this is for a run the caller
        captured into its own graph (drsa_amd_drsa_coop_status; synchronises the stream)."""
        import ctypes
        st = ctypes.c_int(0)
        _capi.call("drsa_amd_drsa_coop_status", self.ptr, self.N, self.d, self.K, ctypes.addressof(st),
                   _capi.stream_ptr(self.buf.device))
        return st.value


def _check_problem(A: torch.Tensor, C: torch.Tensor, U: torch.Tensor, K: int):
    dt = A.dtype if A.dtype in (torch.bfloat16, torch.float16) else torch.float32
    _capi.require_gpu(A, "activation_vecs", dtype=dt)
    _capi.require_gpu(C, "context_vecs", dtype=dt)
    _capi.require_gpu(U, "U")
    if A.dim() != 2 or A.shape != C.shape:
        raise ValueError("activation and context vectors must both be [N, d]")
    d = A.size(1)
    if U.shape != (d, d):
        raise ValueError(f"U must be [{d}, {d}]")
    if K <= 0 or d % K != 0:
        raise ValueError("num_concepts must be a positive divisor of d")


def drsa_objective(A: torch.Tensor, C: torch.Tensor, U: torch.Tensor, K: int,
                   ws: Optional[DrsaWorkspace] = None) -> torch.Tensor:
    """f(U) on device (0-dim fp32 tensor)."""
    _check_problem(A, C, U, K)
    N, d = A.shape
    ws = ws or DrsaWorkspace(N, d, K, A.device)
    _capi.call("drsa_amd_drsa_objective", A.data_ptr(), C.data_ptr(), N, d, K, U.data_ptr(),
               ws.f.data_ptr(), ws.ptr, ws.nbytes, _capi.stream_ptr(A.device))
    return ws.f[0].clone()


def drsa_step(A, C, U, K, ws: Optional[DrsaWorkspace] = None):
    """One optimiser step: returns (U_new, f(U))."""
    _check_problem(A, C, U, K)
    N, d = A.shape
    ws = ws or DrsaWorkspace(N, d, K, A.device)
    U_new = torch.empty_like(U)
    _capi.call("drsa_amd_drsa_step", A.data_ptr(), C.data_ptr(), N, d, K, U.data_ptr(),
               U_new.data_ptr(), ws.f.data_ptr(), ws.ptr, ws.nbytes, _capi.stream_ptr(A.device))
    return U_new, ws.f[0].clone()


def drsa_run(A, C, U0, K: int, steps: int, ws: Optional[DrsaWorkspace] = None,
             use_graph: bool = True):
    """S steps natively. Returns (U_S, trajectory tensor [S+1] on device).  bf16 / fp16 A, C take
    the 16-bit MFMA projection path (drsa_run_joint)."""
    _check_problem(A, C, U0, K)
    if A.dtype in (torch.bfloat16, torch.float16):
        return drsa_run_joint([(A, C, U0, K)], steps, use_graph)[0]
    N, d = A.shape
    ws = ws or DrsaWorkspace(N, d, K, A.device)
    U = U0.detach().clone().contiguous()
    U_tmp = torch.empty_like(U)
    traj = torch.empty(steps + 1, dtype=torch.float32, device=A.device)
    stream = torch.cuda.current_stream(A.device)
    graph = bool(use_graph) and stream.cuda_stream != 0
    _capi.call("drsa_amd_drsa_run", A.data_ptr(), C.data_ptr(), N, d, K, U.data_ptr(),
               U_tmp.data_ptr(), int(steps), traj.data_ptr(), ws.counter.data_ptr(), ws.ptr,
               ws.nbytes, 1 if graph else 0, stream.cuda_stream)
    return U, traj


def drsa_run_joint(problems, steps: int, use_graph: bool = True):
    """Several independent DRSA problems advanced together (C5: the same model's layers j=26 and
    j=33, K=16 each; the reference optimises them one after another, optsubspaces.py:18-23).

    ``problems``: list of (A, C, U0, K) on one device; A, C fp32, or bf16 / fp16 (C5: the
    U-projection GEMM then runs on bf16 / fp16 MFMA with fp32 accumulation).  One hipGraph holds every problem's step
    on its own forked stream (drsa_amd_drsa_run_multi).  Returns [(U_S, trajectory [S+1])]."""
    import ctypes
    if not problems:
        return []
    dev = problems[0][0].device
    keep, structs, outs = [], [], []
    for A, C, U0, K in problems:
        _check_problem(A, C, U0, K)
        if A.device != dev:
            raise ValueError("drsa_run_joint: all problems must live on one device")
        N, d = A.shape
        ws = DrsaWorkspace(N, d, K, dev)
        U = U0.detach().clone().contiguous()
        U_tmp = torch.empty_like(U)
        traj = torch.empty(steps + 1, dtype=torch.float32, device=dev)
        keep += [ws, U_tmp, A, C]
        outs.append((U, traj))
        structs.append(_capi.DrsaProblem(A.data_ptr(), C.data_ptr(), N, d, int(K), U.data_ptr(), U_tmp.data_ptr(),
                                         traj.data_ptr(), ws.counter.data_ptr(), ws.ptr, ws.nbytes,
                                         {torch.bfloat16: 1, torch.float16: 2}.get(A.dtype, 0)))
    arr = (_capi.DrsaProblem * len(structs))(*structs)
    stream = torch.cuda.current_stream(dev)
    graph = bool(use_graph) and stream.cuda_stream != 0
    _capi.call("drsa_amd_drsa_run_multi", len(structs), ctypes.addressof(arr), int(steps), 1 if graph else 0,
               stream.cuda_stream)
    return outs


def batched_geometry(d: int, K: int):
    """(padded d, padded concept width) of a problem: problems sharing it can run batched."""
    dk = d // K
    dkp = 1 << max(0, (dk - 1).bit_length())
    need = max(16, K * dkp)
    return 1 << (need - 1).bit_length(), dkp


def drsa_run_batched(problems, steps: int, blocks: int = 0, use_graph: bool = True):
    """Many independent fp32 DRSA problems of one padded geometry (e.g. the reference's task grid:
    GTZAN classes x layers 19 / 26 / 33 x runs, d = 100 / 128 -> padded 128, concept width 32)
    advanced with one launch per phase for all of them (drsa_amd_drsa_run_batched).  ``blocks``:
    about this many partial workgroups per problem (0 = automatic), each folding whole groups of
    drsa_run's fixed 256-leaf row partition on chip: every result equals drsa_run's bit for bit,
    for any ``blocks``.  Returns [(U_S, trajectory [S+1])]."""
    import ctypes
    if not problems:
        return []
    dev = problems[0][0].device
    keep, structs, outs = [], [], []
    for A, C, U0, K in problems:
        _check_problem(A, C, U0, K)
        if A.dtype != torch.float32:
            raise ValueError("drsa_run_batched: fp32 problems only (use drsa_run_joint for bf16 / fp16)")
        N, d = A.shape
        ws = DrsaWorkspace(N, d, K, dev)
        U = U0.detach().clone().contiguous()
        U_tmp = torch.empty_like(U)
        traj = torch.empty(steps + 1, dtype=torch.float32, device=dev)
        keep += [ws, U_tmp, A, C]
        outs.append((U, traj))
        structs.append(_capi.DrsaProblem(A.data_ptr(), C.data_ptr(), N, d, int(K), U.data_ptr(), U_tmp.data_ptr(),
                                         traj.data_ptr(), ws.counter.data_ptr(), ws.ptr, ws.nbytes, 0))
    arr = (_capi.DrsaProblem * len(structs))(*structs)
    stream = torch.cuda.current_stream(dev)
    graph = bool(use_graph) and stream.cuda_stream != 0
    _capi.call("drsa_amd_drsa_run_batched", len(structs), ctypes.addressof(arr), int(steps), int(blocks),
               1 if graph else 0, stream.cuda_stream)
    return outs


class SubspaceOptimizer:
    """Trains U by gradient ascent + polar retraction (reference drsa.py:15-168)."""

    def __init__(self, U: torch.Tensor, activation_vecs: torch.Tensor, context_vecs: torch.Tensor,
                 path_to_model: str, num_concepts: int = 4,
                 device: str | torch.device = torch.device("cuda")) -> None:
        assert num_concepts > 0, "num_concepts must be a positive number"
        assert U.size(0) % num_concepts == 0, "num_concepts must be a divisor of width (=height) of U"
        self.device = _dev(device)
        self.path_to_model = path_to_model
        self.num_concepts = int(num_concepts)
        self.d_k = U.size(0) // self.num_concepts
        self.U = U.detach().to(self.device, torch.float32).contiguous()
        self.obj_fn = objective_fn
        self.act_vecs = activation_vecs.detach().to(self.device, torch.float32).contiguous()
        self.ctx_vecs = context_vecs.detach().to(self.device, torch.float32).contiguous()
        self._ws = DrsaWorkspace(self.act_vecs.size(0), self.U.size(0), self.num_concepts, self.device)
        self.trajectory: Optional[np.ndarray] = None

    def run(self, steps: int = 2000, save: bool = True) -> None:
        if self.device.index is not None:
            torch.cuda.set_device(self.device)
        side = torch.cuda.Stream(self.device)          # graph capture needs a non-default stream
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            U, traj = drsa_run(self.act_vecs, self.ctx_vecs, self.U, self.num_concepts, steps, self._ws)
        torch.cuda.current_stream(self.device).wait_stream(side)
        self.U = U
        self.trajectory = traj.cpu().numpy()
        if save:
            self.save_model()
            self.save_train_stats([np.asarray(v, dtype=np.float32) for v in self.trajectory])

    @staticmethod
    def obj_val(act_vecs: torch.Tensor, context_vecs: torch.Tensor, U: torch.Tensor,
                obj_fn: Callable = None, num_concepts: int = 4, d_k: int = None) -> torch.Tensor:
        """DRSA objective of U (reference drsa.py:122-155), computed by the HIP kernel.

        ``obj_fn`` must be this module's ``objective_fn`` (the only objective the
        reference defines); ``d_k`` is implied by ``num_concepts``.
        """
        if obj_fn is not None and obj_fn is not objective_fn and getattr(obj_fn, "__name__", "") != "objective_fn":
            raise NotImplementedError("obj_val: only the DRSA objective_fn is implemented on device")
        if d_k is not None and d_k * num_concepts != U.size(0):
            raise ValueError("d_k * num_concepts must equal d")
        return drsa_objective(act_vecs.detach().contiguous(), context_vecs.detach().contiguous(),
                              U.detach().contiguous(), num_concepts)

    def save_train_stats(self, obj_arr: List[np.ndarray]) -> None:
        import pandas as pd
        pd.DataFrame({"loss": obj_arr}).to_csv(os.path.join(self.path_to_model, "train_stats.csv"))

    def save_model(self) -> None:
        with open(os.path.join(self.path_to_model, "projection_matrix.pkl"), "wb") as fh:
            pickle.dump(self.U.detach().cpu().numpy(), fh)


def generalized_fmean(x: torch.Tensor, p: float = 0.5) -> torch.Tensor:
    """Power mean over dim 0 (reference drsa.py:171-182); a tensor-expression helper."""
    return torch.pow(torch.mean(torch.pow(x, p), dim=0), 1 / p)


def objective_fn(input: torch.Tensor) -> torch.Tensor:
    """Soft-min over concepts of soft-max over points (reference drsa.py:224-238)."""
    return generalized_fmean(generalized_fmean(input, 2), 0.5)


@torch.no_grad()
def project_grad(gradient: torch.Tensor, U: torch.Tensor) -> torch.Tensor:
    """Tangent-space projection (reference drsa.py:185-198, unused by the reference)."""
    return gradient - (U.T @ gradient) @ U.T


@torch.no_grad()
def orthogonalize(U: torch.Tensor) -> torch.Tensor:
    """Polar factor U (UᵀU)^{-1/2} (reference drsa.py:201-221), on device (Newton–Schulz)."""
    _capi.require_gpu(U, "U")
    d = U.size(0)
    if U.shape != (d, d):
        raise ValueError("orthogonalize expects a square matrix")
    out = torch.empty_like(U)
    _capi.call("drsa_amd_polar", U.data_ptr(), d, out.data_ptr(), None, _capi.stream_ptr(U.device))
    return out


def initial_projections(d: int, runs: int, seed: int = 42) -> List[np.ndarray]:
    """drsa.main's U schedule (drsa.py:265-285): ortho_group.rvs(d) after np.random.seed(seed),
    then per run a column permutation of the previous run's initial U (compounding)."""
    from scipy.stats import ortho_group
    np.random.seed(seed)
    U = ortho_group.rvs(d)
    out = []
    for _ in range(runs):
        mask = np.random.permutation(d)
        U = np.asarray(U)[:, mask]
        out.append(U)
    return out


def main(activation_vecs: torch.Tensor, context_vecs: torch.Tensor, model_root: str,
         num_concepts: int = 4, steps: int = 2000, runs: int = 3, seed: int = 42,
         device: str | torch.device = torch.device("cuda")) -> None:
    """Several DRSA runs from permuted random orthogonal starts (reference drsa.py:241-301)."""
    device = _dev(device)
    d = activation_vecs.size(-1)
    print(f"Starting DRSA training on device {device} ...")
    for run, U in enumerate(initial_projections(d, runs, seed), start=1):
        path = os.path.join(model_root, f"run{run}")
        os.makedirs(path, exist_ok=True)
        Ut = torch.tensor(U, dtype=activation_vecs.dtype, device=device)
        print("-" * 20, f"\nStarting RUN {run}")
        opt = SubspaceOptimizer(Ut, activation_vecs, context_vecs, path, num_concepts=num_concepts,
                                device=device)
        opt.run(steps=steps)
    print("Done!")
