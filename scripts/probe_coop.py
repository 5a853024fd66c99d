"""Phase stamps of the cooperative DP = 128 finish (drsa_finish_coop_kernel) in a C5-shaped
drsa_run (N = 20 000, d = 128, K = 16).  Needs the stamp build:
  python scripts/build_variant.py coopstamp drsa_step.hip -DDRSA_COOP_STAMP
  DRSA_AMD_LIB=drsa_audio_amd/lib/exp/coopstamp.so python scripts/probe_coop.py"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drsa_audio_amd import _capi  # noqa: E402
from drsa_audio_amd.utils.synthetic import drsa_inputs  # noqa: E402
from drsa_audio_amd.xai.drsa.drsa import drsa_run  # noqa: E402

dev = torch.device("cuda")
A, C = drsa_inputs(20000, 128, 5)
U0 = np.linalg.qr(np.random.default_rng(5).standard_normal((128, 128)))[0].astype(np.float32)
Ag, Cg, Ug = (torch.from_numpy(v).to(dev) for v in (A, C, U0))
out = {}
for steps in (1, 7):
    drsa_run(Ag, Cg, Ug, 16, steps, use_graph=False)
    torch.cuda.synchronize()
    st = (ctypes.c_ulonglong * (8 * 64))()
    _capi.lib().drsa_amd_debug_coop_stamps(st)
    a = np.array(st, dtype=np.float64).reshape(8, 64)
    t0 = a[:, 0].min()
    rows = {}
    for j in range(8):
        rows[j] = {k: round((a[j, k] - t0) / 1e3, 2) for k in range(64) if a[j, k] >= t0 and a[j, k] > 0}
    out[f"steps{steps}"] = rows   # kilocycles since the first workgroup's start
print(json.dumps(out))
