"""Task-parallel DRSA over the reference's problem grid, drop-in for the
driver ``cxai/xai/drsa/cluster/optsubspaces.py``.

The reference optimises every (class, layer) dataset one after the other, each with
``drsa.main(A, C, root/{class}/layer{L}, num_concepts, steps=5000, runs=3, seed=42)``
(optsubspaces.py:17-23: 10 GTZAN classes x layers [19, 26, 33] x 3 runs = 90 independent
problems).  Here the grid of (class, layer, run) tasks is spread over the ranks of the process
group (one process per GPU) by longest-processing-time assignment (cost ~ N * padded d^2); each
rank advances all of its tasks together, <= ``max_joint`` at a time, in one hipGraph per two
steps (``drsa_run_joint`` -> ``drsa_amd_drsa_run_multi``), so the single-workgroup polar of one
problem overlaps the partials of the others.  There is no collective on the data path: the only
exchange is a final ``all_gather_object`` of the per-task objectives.

Every task writes what ``drsa.main`` writes for its run (drsa.py:157-168):
``{model_root}/{class}/layer{L}/run{r}/projection_matrix.pkl`` and ``train_stats.csv``; the run's
initial U is drsa.main's compounding column permutation of ``ortho_group.rvs(d)`` after
``np.random.seed(seed)`` (drsa.py:265-285), identical to the sequential reference.

``runner`` is pluggable so the orchestration is tested on CPU with gloo (tests/test_dist_cpu.py);
the product runner is the HIP one.
"""
from __future__ import annotations

import os
import pickle
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

# optsubspaces.py conf 1: GTZAN classes x VGGish-BN DRSA layers (getdrsadata.py:119)
GTZAN_CLASSES = ("pop", "metal", "disco", "blues", "reggae", "classical", "rock", "hiphop", "country", "jazz")
GTZAN_LAYERS = (19, 26, 33)


@dataclass(frozen=True)
class Task:
    sample_class: str
    layer_idx: int
    run: int            # 1-based, as drsa.main's run{r}
    d: int
    N: int

    @property
    def cost(self) -> int:
        dp = 1 << max(5, (self.d - 1).bit_length())      # kernels run d padded to a power of two
        return self.N * dp * dp

    @property
    def key(self) -> Tuple[str, int, int]:
        return (self.sample_class, self.layer_idx, self.run)


def problem_grid(shapes: Dict[Tuple[str, int], Tuple[int, int]], runs: int = 3) -> List[Task]:
    """All (class, layer, run) tasks; ``shapes[(class, layer)] = (N, d)``.  Order: the
    reference's loop order (class, layer, run)."""
    return [Task(c, l, r, d, N) for (c, l), (N, d) in shapes.items() for r in range(1, runs + 1)]


def assign(tasks: Sequence[Task], world: int) -> List[List[Task]]:
    """Longest-processing-time assignment: tasks by descending cost (ties: grid order), each to
    the least-loaded rank (ties: lowest rank).  Deterministic, so every rank derives the same
    plan without communicating."""
    order = sorted(range(len(tasks)), key=lambda i: (-tasks[i].cost, i))
    load = [0] * world
    out: List[List[Task]] = [[] for _ in range(world)]
    for i in order:
        r = min(range(world), key=lambda q: (load[q], q))
        out[r].append(tasks[i])
        load[r] += tasks[i].cost
    pos = {t.key: i for i, t in enumerate(tasks)}
    for r in range(world):
        out[r].sort(key=lambda t: pos[t.key])
    return out


def hip_runner(problems, steps: int):
    """Product runner.  Problems sharing one padded geometry run batched -- one launch per phase
    for all of them (drsa_run_batched); mixed geometries or 16-bit inputs advance together in one
    hipGraph of per-problem chains (drsa_run_joint)."""
    from ..drsa import batched_geometry, drsa_run_batched, drsa_run_joint
    dev = problems[0][0].device
    side = torch.cuda.Stream(dev)             # graph capture needs a non-default stream
    side.wait_stream(torch.cuda.current_stream(dev))
    geoms = {batched_geometry(A.size(1), K) for A, _, _, K in problems}
    fp32 = all(A.dtype == torch.float32 for A, _, _, _ in problems)
    with torch.cuda.stream(side):
        if len(geoms) == 1 and fp32:
            # the batched partial folds whole groups of drsa_run's fixed 256-leaf row partition
            # per workgroup, so the fp32 summation order is drsa_run's whatever the workgroup
            # count, the tasks sharing the launch, the world size or the LPT plan: grid results
            # equal drsa.main's bit for bit
            out = drsa_run_batched(problems, steps)
        else:
            out = drsa_run_joint(problems, steps)
    torch.cuda.current_stream(dev).wait_stream(side)
    return out


def _write_run(path: str, U: np.ndarray, traj: np.ndarray) -> None:
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "projection_matrix.pkl"), "wb") as fh:
        pickle.dump(np.asarray(U, dtype=np.float32), fh)
    import pandas as pd
    pd.DataFrame({"loss": [np.asarray(v, dtype=np.float32) for v in traj]}).to_csv(
        os.path.join(path, "train_stats.csv"))


def optimize_grid(datasets: Dict[Tuple[str, int], Tuple[torch.Tensor, torch.Tensor]], model_root: Optional[str],
                  num_concepts: int = 4, steps: int = 5000, runs: int = 3, seed: int = 42, device=None,
                  group=None, runner: Optional[Callable] = None, max_joint: int = 128,
                  dtype: torch.dtype = torch.float32) -> Dict[Tuple[str, int, int], Dict]:
    """Optimise every (class, layer, run) DRSA problem of ``datasets`` over the process group.

    ``datasets[(class, layer)] = (A, C)``, normalised [N, d] vectors (``load_and_normalize_data``);
    every rank passes the same dict (host or device tensors: a rank moves only its own tasks'
    data to its GPU).  With ``model_root`` the files of each run are written by the rank that
    ran it.  Returns on every rank ``{(class, layer, run): {"objective": f_S, "rank": r,
    "trajectory": ..(own tasks only)}}``."""
    from ..drsa import initial_projections
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    runner = runner or hip_runner
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if runner is hip_runner else torch.device("cpu")
    shapes = {k: (int(A.size(0)), int(A.size(1))) for k, (A, C) in datasets.items()}
    tasks = problem_grid(shapes, runs)
    mine = assign(tasks, world)[rank]
    # drsa.main's U schedule re-seeds per dataset (drsa.py:265), so it depends on d only
    by_d = {d: initial_projections(d, runs, seed) for d in sorted({d for _, d in shapes.values()})}
    U0s = {k: by_d[d] for k, (N, d) in shapes.items()}
    local: Dict[Tuple[str, int, int], Dict] = {}
    dev_data: Dict[Tuple[str, int], Tuple[torch.Tensor, torch.Tensor]] = {}
    # tasks of one padded geometry run batched (one launch per phase for all of them): group first
    from ..drsa import batched_geometry
    by_geom: Dict[Tuple[int, int], List[Task]] = {}
    for t in mine:
        by_geom.setdefault(batched_geometry(t.d, num_concepts), []).append(t)
    chunks = [grp[i:i + max(1, max_joint)] for grp in by_geom.values() for i in range(0, len(grp), max(1, max_joint))]
    for chunk in chunks:
        probs = []
        for t in chunk:
            k = (t.sample_class, t.layer_idx)
            if k not in dev_data:
                A, C = datasets[k]
                dev_data[k] = (A.to(device, dtype).contiguous(), C.to(device, dtype).contiguous())
            A, C = dev_data[k]
            U0 = torch.tensor(np.ascontiguousarray(U0s[k][t.run - 1]), dtype=torch.float32, device=device)  # drsa.py:285
            probs.append((A, C, U0, num_concepts))
        for t, (U, traj) in zip(chunk, runner(probs, steps)):
            U_np = U.detach().cpu().numpy()
            traj_np = traj.detach().cpu().numpy() if torch.is_tensor(traj) else np.asarray(traj)
            if model_root is not None:
                _write_run(os.path.join(model_root, t.sample_class, f"layer{t.layer_idx}", f"run{t.run}"), U_np, traj_np)
            local[t.key] = {"objective": float(traj_np[-1]), "rank": rank, "trajectory": traj_np, "U": U_np}
    summary = {k: {"objective": v["objective"], "rank": v["rank"]} for k, v in local.items()}
    if dist.is_initialized() and world > 1:
        allv: List[Optional[Dict]] = [None] * world
        dist.all_gather_object(allv, summary, group=group)
        for part in allv:
            for k, v in part.items():
                summary[k] = v
    for k, v in local.items():
        summary[k] = v
    return summary


def main(conf: int = 1, path_to_data: str = "/input-data", path_to_models: str = ".", steps: int = 5000,
         device=None) -> Dict:
    """optsubspaces.main(args) (optsubspaces.py:8-47) on the process group: conf 1 = GTZAN 10
    classes x layers [19, 26, 33], K = 4; conf 2 / 3 = the VGGish 4c / 2c sets, layers [9, 14],
    K = 2.  Reads ``{path_to_data}/.../dataset_layer{L}.pkl`` (getdrsadata.save_data format)."""
    from .getdrsadata import load_and_normalize_data
    if conf == 1:
        classes, layers, K, sub = GTZAN_CLASSES, GTZAN_LAYERS, 4, "gtzan/1700_big_norm_20/{c}"
    elif conf == 2:
        classes, layers, K, sub = ("class1", "class2", "class3", "class4"), (9, 14), 2, "{c}"
    else:
        classes, layers, K, sub = ("class1", "class2"), (9, 14), 2, "{c}"
    device = device or torch.device("cuda", torch.cuda.current_device())
    data = {}
    for c in classes:
        for l in layers:
            # normalised on the GPU, then kept on the host: optimize_grid moves only this rank's
            # tasks' datasets to the device
            a, cv = load_and_normalize_data(
                os.path.join(path_to_data, sub.format(c=c), f"dataset_layer{l}.pkl"), device=device)
            data[(c, l)] = (a.cpu(), cv.cpu())
            del a, cv
    return optimize_grid(data, path_to_models, num_concepts=K, steps=steps, runs=3, seed=42, device=device)
