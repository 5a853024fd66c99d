#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the features.3 backward conv.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $c --output-format csv \
    -d $O/$c -o run -- python scripts/run_conv_bwd3.py > $O/$c.log 2>&1
done
