"""Phase stamps of every workgroup of the GTZAN conv_bwd:features.3 shape (B = 512 x 4 clones, 32 ->
32 at 64 x 64, pool-sparse g): where the MFMA pipe idles.  Needs the stamp build:
  python scripts/build_variant.py convstamp conv_bwd_b.hip -DDRSA_CONV_STAMP
  DRSA_AMD_LIB=drsa_audio_amd/lib/exp/convstamp.so python scripts/probe_conv_phases.py
Slots per workgroup (s_memtime, shader cycles): 0 start, 1 + 2c chunk c staged, 2 + 2c chunk c's MFMAs
issued (wave 0), 13 end, 14 HW_ID, 15 XCC_ID."""
import collections
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drsa_audio_amd import _capi  # noqa: E402

dev = torch.device("cuda")
Bs, clones = 512, 4
Bq = Bs * clones
g = torch.randn(Bq, 32, 32, 32, device=dev)
amax = torch.randint(0, 4, (Bs, 32, 32, 32), device=dev, dtype=torch.uint8)
w = torch.randn(1, 9 * 32, 32, device=dev)
x = torch.rand(Bs, 32, 64, 64, device=dev)
den = torch.rand(Bs, 32, 64, 64, device=dev) + 0.5
out = torch.empty(Bq, 32, 64, 64, device=dev)
tiles = 16
st = torch.zeros(Bq * tiles * 16, dtype=torch.int64, device=dev)
s = _capi.stream_ptr()


def run():
    _capi.call("drsa_amd_conv_bwd", g.data_ptr(), amax.data_ptr(), w.data_ptr(), x.data_ptr(), den.data_ptr(),
               out.data_ptr(), Bq, clones, 32, 32, 64, 64, 1, 1, 1, 1e-7, s)


for _ in range(3):
    run()
_capi.lib().drsa_amd_debug_conv_stamps(ctypes.c_void_p(st.data_ptr()))
run()
torch.cuda.synchronize()
a = st.view(Bq * tiles, 16).cpu().numpy().astype(np.int64)
NCH = 4
hw, xcc = a[:, 14], a[:, 15]
cu = (xcc << 8) | (((hw >> 13) & 7) << 4) | ((hw >> 8) & 15)   # xcc, se, cu
life = a[:, 13] - a[:, 0]

first = a[:, 1] - a[:, 0]                                  # first chunk loaded + staged
# first chunk split: 11 loads issued, 9 past the first barrier, 10 stored (loads landed)
f_issue, f_bar1, f_store, f_bar2 = a[:, 11] - a[:, 0], a[:, 9] - a[:, 11], a[:, 10] - a[:, 9], a[:, 1] - a[:, 10]
mf = [a[:, 2 + 2 * c] - a[:, 1 + 2 * c] for c in range(NCH)]          # chunk c MFMA issue span
stg = [a[:, 1 + 2 * c] - a[:, 2 * c] for c in range(1, NCH)]          # chunk c staging (after c-1's MFMAs)
epi = a[:, 13] - a[:, 2 * NCH]
res = {"workgroups": int(len(a)), "cus": int(len(set(cu.tolist()))),
       "median_cycles": {"lifetime": float(np.median(life)), "first_stage": float(np.median(first)),
                         **{f"mfma_{c}": float(np.median(mf[c])) for c in range(NCH)},
                         **{f"stage_{c + 1}": float(np.median(stg[c])) for c in range(NCH - 1)},
                         "epilogue": float(np.median(epi)),
                       "first_issue": float(np.median(f_issue)), "first_barrier1": float(np.median(f_bar1)),
                       "first_store_wait": float(np.median(f_store)), "first_barrier2": float(np.median(f_bar2))},
       "first_store_wait_pct": {str(q): float(np.percentile(f_store, q)) for q in (10, 25, 50, 75, 90, 99)}}
# per CU: concurrency (workgroups alive) over time and the fraction of time with k workgroups in an
# MFMA span
by = collections.defaultdict(list)
for i in range(len(a)):
    by[int(cu[i])].append(i)
conc, busyk = [], collections.Counter()
for c, idx in list(by.items())[:32]:
    ev = []
    for i in idx:
        ev += [(a[i, 0], 1, 0), (a[i, 13], -1, 0)]
        for k in range(NCH):
            ev += [(a[i, 1 + 2 * k], 0, 1), (a[i, 2 + 2 * k], 0, -1)]
    ev.sort()
    alive = inm = 0
    t0 = ev[0][0]
    for t, da, dm in ev:
        busyk[inm] += t - t0
        conc.append((alive, t - t0))
        alive += da
        inm += dm
        t0 = t
tot = sum(busyk.values())
res["time_share_by_workgroups_in_mfma_span"] = {k: round(v / tot, 3) for k, v in sorted(busyk.items())}
ca = collections.Counter()
for k, dt in conc:
    ca[k] += dt
tc = sum(ca.values())
res["time_share_by_workgroups_alive"] = {k: round(v / tc, 3) for k, v in sorted(ca.items())}
print(json.dumps(res, indent=1))

# MFMA spans bucketed by how many OTHER workgroups of the same CU were in an MFMA span meanwhile
# (time-averaged): if a lone workgroup's span is near 72 MFMAs x 64 cycles = 4.6k, one wave per SIMD
# keeps the pipe busy and the idle time comes from phases with no MFMA work; if it stays long, the
# single wave's own issue (operand latency) is the limit
spans = collections.defaultdict(list)
for c, idx in list(by.items())[:64]:
    iv = [(a[i, 1 + 2 * k], a[i, 2 + 2 * k], i) for i in idx for k in range(NCH - 1)]
    for s0, s1, i in iv:
        if s1 <= s0:
            continue
        ov = 0
        for t0_, t1_, j in iv:
            if j == i:
                continue
            ov += max(0, min(s1, t1_) - max(s0, t0_))
        spans[int(round(ov / (s1 - s0)))].append(s1 - s0)
res["mfma_span_cycles_by_concurrent_workgroups"] = {k: {"n": len(v), "median": float(np.median(v))}
                                                    for k, v in sorted(spans.items())}
print(json.dumps({"mfma_span_cycles_by_concurrent_workgroups": res["mfma_span_cycles_by_concurrent_workgroups"]}))
