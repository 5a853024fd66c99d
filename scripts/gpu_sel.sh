#!/bin/bash
# Selected GPU tests + headline bench legs.  Usage: gpu_sel.sh <tag> "<pytest selection>" [bench args]
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
SEL=$2
shift 2
mkdir -p $O
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_sel.log 2>&1
timeout -k 10 400 python bench.py --no-cpu-baseline "$@" > $O/bench.json 2> $O/bench.err
