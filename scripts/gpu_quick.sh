#!/bin/bash
# Quick GPU pass: parity tests + bench (no profiling).  Usage: gpu_quick.sh <tag> [bench args]
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift
mkdir -p $O
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1
timeout -k 10 400 python bench.py --no-cpu-baseline "$@" > $O/bench.json 2> $O/bench.err
