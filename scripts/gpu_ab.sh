#!/bin/bash
# Selected GPU tests, then the headline bench under two environments (A/B on one box).
# Usage: gpu_ab.sh <tag> "<pytest targets>" "<env A>" "<env B>" [bench args...]
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1; T=$2; EA=$3; EB=$4; shift 4
mkdir -p $O
if [ -n "$T" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $T > $O/pytest_gpu.log 2>&1
fi
for i in 1 2; do
  env $EA timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/bench_A$i.json 2> $O/bench_A$i.err
  env $EB timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/bench_B$i.json 2> $O/bench_B$i.err
done
python - "$O" <<'PY'
import json, sys, glob, os
o = sys.argv[1]
for f in sorted(glob.glob(os.path.join(o, "bench_*.json"))):
    try:
        d = json.load(open(f))
    except Exception as e:
        print(f, "unreadable", e); continue
    ks = d.get("kernels", {})
    top = sorted(ks.items(), key=lambda kv: -kv[1]["avg_ms"])[:8]
    print(os.path.basename(f), f"{d['value']:.0f}/s {d['ms_per_step']:.3f} ms", " ".join(f"{k}={v['avg_ms']:.3f}" for k, v in top))
PY
