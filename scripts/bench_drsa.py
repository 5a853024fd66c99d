"""DRSA-only timing: C3 (N=20000, d=64, K=4) drsa_run and the C5 joint run (2 x d=128, K=16),
via bench.py's helpers, plus the Newton-Schulz iteration counts of one finish at each size.
python scripts/bench_drsa.py [steps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from drsa_audio_amd import _capi  # noqa: E402
from drsa_audio_amd.xai.drsa.drsa import DrsaWorkspace  # noqa: E402
from drsa_audio_amd.utils.synthetic import drsa_inputs  # noqa: E402


def ns_iters(dev, N, d, K, seed):
    A, C = drsa_inputs(N, d, seed)
    U0 = np.linalg.qr(np.random.default_rng(seed).standard_normal((d, d)))[0].astype(np.float32)
    Ag, Cg, Ug = (torch.from_numpy(v).to(dev) for v in (A, C, U0))
    ws = DrsaWorkspace(N, d, K, dev)
    st = _capi.stream_ptr(dev)
    out, its = [], torch.zeros(1, dtype=torch.int32, device=dev)
    U = Ug
    for _ in range(5):
        _capi.call("drsa_amd_drsa_partial", Ag.data_ptr(), Cg.data_ptr(), N, d, K, U.data_ptr(), ws.gs.data_ptr(),
                   ws.ptr, ws.nbytes, st)
        Un = torch.empty_like(U)
        _capi.call("drsa_amd_drsa_finish", ws.gs.data_ptr(), N, d, K, U.data_ptr(), Un.data_ptr(), ws.f.data_ptr(), 0,
                   its.data_ptr(), st)
        out.append(int(its.item()))
        U = Un
    return out


steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
dev = torch.device("cuda", 0)
out = {"drsa_c3": bench.drsa_bench(dev, steps=steps), "drsa_joint_c5": bench.drsa_joint_bench(dev, steps=steps),
       "ns_iters_c3": ns_iters(dev, 20000, 64, 4, 3), "ns_iters_d128": ns_iters(dev, 20000, 128, 16, 26),
       "ns_iters_d100": ns_iters(dev, 20000, 100, 4, 13)}
print(json.dumps(out, indent=1))
