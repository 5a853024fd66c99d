"""One RCCL rank (world size 1): the sharded DRSA loops with the captured step graph vs eagerly
(DRSA_AMD_SHARDED_GRAPH=0); C4 shape (d=64, K=8, 20000 rows) and the C5 joint pair (d=128, K=16)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import numpy as np
import torch
import torch.distributed as dist

from drsa_audio_amd.utils.synthetic import drsa_inputs

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
from drsa_audio_amd.xai.drsa import distributed as D

A, C = drsa_inputs(20000, 64, 1)
Ag, Cg = torch.from_numpy(A).to(dev), torch.from_numpy(C).to(dev)
U0 = torch.linalg.qr(torch.randn(64, 64, dtype=torch.float64))[0].float().to(dev)
g = torch.Generator().manual_seed(5)
probs = []
for p in range(2):
    A5, C5 = drsa_inputs(20000, 128, 200 + p)
    U5 = torch.linalg.qr(torch.randn(128, 128, generator=g, dtype=torch.float64))[0].float()
    probs.append((torch.from_numpy(A5).to(dev), torch.from_numpy(C5).to(dev), U5.to(dev), 16))
out = {}
for mode in ("0", "1"):
    os.environ["DRSA_AMD_SHARDED_GRAPH"] = mode
    res = {}
    for name, fn, steps in (("c4_fused", lambda s: D.sharded_run(Ag, Cg, U0, 8, s), 200),
                            ("c5_joint", lambda s: D.sharded_run_joint(probs, s), 100)):
        fn(4)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn(steps)
        torch.cuda.synchronize()
        res[name] = (time.perf_counter() - t0) / steps * 1e3
    out["graph" if mode == "1" else "eager"] = res
out["stats"] = D.STATS
print(json.dumps(out))
dist.destroy_process_group()
