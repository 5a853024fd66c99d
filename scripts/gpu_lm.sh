#!/bin/bash
# log-mel front end: parity tests + micro-bench + rocprofv3 kernel stats.  Usage: gpu_lm.sh <tag>
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_logmel_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1
timeout -k 10 120 python scripts/bench_frontend.py > $O/b.json 2> $O/b.err
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python scripts/bench_frontend.py > /dev/null 2>&1
tail -2 $O/t.log; cat $O/b.json
