"""A/B the headline bench over environment toggles: python scripts/ab_env.py NAME=v1,v2 [...] -- bench args.
Prints value and the per-tag kernel times for each setting (one bench process per setting)."""
import itertools
import json
import os
import subprocess
import sys

args = sys.argv[1:]
sep = args.index("--") if "--" in args else len(args)
toggles = [a.split("=", 1) for a in args[:sep]]
bench_args = args[sep + 1:]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for combo in itertools.product(*[v.split(",") for _, v in toggles]):
    env = dict(os.environ)
    for (k, _), v in zip(toggles, combo):
        env[k] = v
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--no-cpu-baseline", "--no-drsa", *bench_args],
                       capture_output=True, text=True, env=env, timeout=600)
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    if not line:
        print(combo, "FAILED", r.stderr[-2000:])
        continue
    b = json.loads(line[-1])
    ks = {k: round(v["avg_ms"], 4) for k, v in b["kernels"].items()}
    print(json.dumps({"env": dict(zip([k for k, _ in toggles], combo)), "value": round(b["value"]),
                      "ms_per_step": round(b["ms_per_step"], 4), "kernels": ks}))
