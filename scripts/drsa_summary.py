"""Summarise a gpu_drsa.sh output directory: test results, DRSA timings, per-kernel rocprof stats."""
import csv
import json
import os
import re
import sys

d = sys.argv[1]
for f in ("pytest_drsa.log", "pytest_rest.log"):
    p = os.path.join(d, f)
    if os.path.exists(p):
        for line in open(p):
            if re.search(r"passed|failed|error|^\[(c3|c4|d100)\]", line):
                print(f, line.rstrip()[:200])
p = os.path.join(d, "bench_drsa.json")
if os.path.exists(p) and os.path.getsize(p):
    b = json.load(open(p))
    print("C3 ms/step", b["drsa_c3"]["ms_per_step"], "| C5 joint", b["drsa_joint_c5"]["ms_per_joint_step"],
          "bf16", b["drsa_joint_c5"]["bf16"]["ms_per_joint_step"], "| NS iters", b.get("ns_iters_c3"),
          b.get("ns_iters_d128"), b.get("ns_iters_d100"))
p = os.path.join(d, "prof", "run_kernel_stats.csv")
if os.path.exists(p):
    for r in csv.DictReader(open(p)):
        n = r["Name"]
        if any(k in n for k in sys.argv[2:] or ("drsa", "polar", "subrel")):
            print(f"{n[:72]:72s} calls {r['Calls']:>6} avg {float(r['AverageNs'])/1000:8.2f}us "
                  f"min {float(r['MinNs'])/1000:8.2f} max {float(r['MaxNs'])/1000:8.2f}")
