#!/bin/bash
# Selected GPU tests then an optional bench.  Usage: gpu_sel.sh <tag> "<pytest targets>" [bench args...]
# (bench is skipped when no bench args are given; pass "-" for a default bench run)
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1; T=$2; shift 2
mkdir -p $O
if [ -n "$T" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $T > $O/pytest_gpu.log 2>&1
fi
if [ $# -gt 0 ]; then
  [ "$1" = "-" ] && shift
  timeout -k 10 500 python bench.py "$@" > $O/bench.json 2> $O/bench.err
fi
