"""Summarise scripts/ab_bench.sh output: ms/step and per-tag HIP-event ms of each variant and repeat.
python scripts/ab_summary.py gpurun_out/<tag> [tag-regex]"""
import glob
import json
import os
import re
import sys

d = sys.argv[1]
rx = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"conv_bwd|conv_fwd:features\.[36]|projection|first_layer")
rows = {}
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    try:
        j = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception:
        continue
    name = os.path.basename(f)[:-5]
    rows[name] = {"step": j["ms_per_step"], **{k: v["avg_ms"] for k, v in j["kernels"].items() if rx.search(k)}}
tags = sorted({k for r in rows.values() for k in r if k != "step"})
print(f"{'variant':>12} {'step':>7} " + " ".join(f"{t[-18:]:>18}" for t in tags))
for n, r in rows.items():
    print(f"{n:>12} {r['step']:7.3f} " + " ".join(f"{r.get(t, float('nan')):18.4f}" for t in tags))
