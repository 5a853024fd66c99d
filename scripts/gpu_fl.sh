#!/bin/bash
# first-layer backward: LRP parity tests + A/B micro-bench.  Usage: gpu_fl.sh <tag> [variant...]
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_lrp_gpu.py tests/test_engine_gpu.py tests/test_logmel_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
bash scripts/ab_lib.sh $(basename $O)_ab ${AB_SCRIPT:-scripts/bench_first_layer.py} "$@"
