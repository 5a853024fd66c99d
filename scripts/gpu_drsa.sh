#!/bin/bash
# DRSA-focused GPU pass: DRSA/R11 parity tests, the rest of the GPU suite, DRSA timings and a
# rocprofv3 kernel-trace summary of the DRSA timing run.  Usage: gpu_drsa.sh <tag>
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_drsa_gpu.py tests/test_drsa_long_gpu.py tests/test_subrel.py -s > $O/pytest_drsa.log 2>&1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests \
  --deselect tests/test_drsa_gpu.py --deselect tests/test_drsa_long_gpu.py --deselect tests/test_subrel.py \
  > $O/pytest_rest.log 2>&1
timeout -k 10 300 python scripts/bench_drsa.py 200 > $O/bench_drsa.json 2> $O/bench_drsa.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python scripts/bench_drsa.py 100 > $O/prof_drsa.json 2> $O/prof_drsa.err
