"""Per-phase clock cycles of logmel800_kernel (a build with -DLF_PROFILE, selected by DRSA_AMD_LIB).
  python scripts/build_variant.py lfprof logmel.hip -DLF_PROFILE
  DRSA_AMD_LIB=drsa_audio_amd/lib/exp/lfprof.so python scripts/logmel_phases.py"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import numpy as np
import torch

import logmel_ref
from drsa_audio_amd import _capi
from drsa_audio_amd.utils.dataloading import Loader

dev = torch.device("cuda")
songs = torch.from_numpy(logmel_ref.synthetic_songs(64, seed=3)).to(dev)
ld = Loader("gtzan", device=dev)
for _ in range(3):
    ld.load_songs(songs)
torch.cuda.synchronize()
lib = _capi.load()
WAVES = int(os.environ.get("LF_WAVES", "8"))
n = 512 * WAVES * 8
buf = np.zeros(n, dtype=np.uint64)
assert lib.drsa_amd_logmel_prof(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(n)) == 0
c = buf.reshape(512, WAVES, 8).astype(np.float64)
names = ["init", "load+window", "dftA+twiddle", "transpose", "dftB", "split+|X|", "mel", "log pass"]
tot = c.sum(axis=2).mean()
print(json.dumps({"cycles_per_wave_mean": {k: float(v) for k, v in zip(names, c.mean(axis=(0, 1)))},
                  "total_cycles_per_block": float(tot)}, indent=1))
