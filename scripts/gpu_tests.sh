#!/bin/bash
# Full GPU parity suite with per-test timeouts.  Usage: gpu_tests.sh <tag> [pytest args]
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -s tests "$@" > $O/pytest_gpu.log 2>&1
