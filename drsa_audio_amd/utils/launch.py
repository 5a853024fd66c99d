"""One process per GPU, launched from a parent that never touches the GPU.

``bench.py --gpus N`` (and any script) calls ``maybe_launch(N)`` first thing: when the process was
not started by ``torch.distributed.run`` (no ``WORLD_SIZE`` in the environment) and N > 1, the
parent spawns N children of the same command line with ``RANK`` / ``LOCAL_RANK`` / ``WORLD_SIZE``
/ ``LOCAL_WORLD_SIZE`` / ``MASTER_ADDR=127.0.0.1`` / ``MASTER_PORT`` set, forwards rank 0's stdout,
waits, and exits with the first failing child's code.  Children are started as new processes
(``subprocess``), never by ``exec`` from a process that has initialised the GPU; the parent only
counts devices (``torch.cuda.device_count()``, which does not initialise HIP).

Each child then binds ``cuda:LOCAL_RANK`` (``init_distributed``) and joins the ``nccl`` (= RCCL)
process group with ``device_id``, or ``gloo`` when asked (CPU tests, one-GPU rehearsals).
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import time
from typing import List, Optional, Sequence


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn(nprocs: int, argv: Sequence[str], env: Optional[dict] = None, timeout: Optional[float] = None,
          stdout_rank: int = 0) -> int:
    """Run ``argv`` as ``nprocs`` ranks.  Rank ``stdout_rank``'s stdout goes to ours, every other
    rank's stdout to our stderr; stderr is inherited.  Returns 0, or the first nonzero exit code
    (the remaining ranks are terminated, by handle)."""
    port = free_port()
    base = dict(os.environ if env is None else env)
    procs: List[subprocess.Popen] = []
    for r in range(nprocs):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nprocs), LOCAL_WORLD_SIZE=str(nprocs),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GROUP_RANK="0")
        procs.append(subprocess.Popen(list(argv), env=e, stdout=None if r == stdout_rank else sys.stderr))
    t0 = time.monotonic()
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            if timeout is not None and time.monotonic() - t0 > timeout:
                rc = 124
                break
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                if rc:
                    p.terminate()
                try:
                    p.wait(timeout=30 if rc else None)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
    return rc


def maybe_launch(nprocs: int, one_device: bool = False) -> None:
    """If this process should fan out into ``nprocs`` ranks, do it and exit with their status."""
    if nprocs <= 1 or "WORLD_SIZE" in os.environ:
        return
    if not one_device:
        import torch
        n = torch.cuda.device_count()          # does not initialise HIP on this stack
        if n < nprocs:
            raise SystemExit(f"--gpus {nprocs}: only {n} GPU(s) visible (set DRSA_BENCH_ONE_DEVICE=1 for a "
                             "one-device rehearsal)")
    sys.stdout.flush()
    sys.exit(spawn(nprocs, [sys.executable, "-u"] + sys.argv))


def init_distributed(backend: Optional[str] = None, one_device: bool = False):
    """Join the process group described by the environment.  Returns (world, rank, device)."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if one_device else int(os.environ.get("LOCAL_RANK", "0"))
    backend = backend or "nccl"
    if backend == "gloo" and not torch.cuda.is_available():
        device = torch.device("cpu")
    else:
        device = torch.device("cuda", local)
        torch.cuda.set_device(device)
    if world > 1 and not dist.is_initialized():
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)
    return world, rank, device
