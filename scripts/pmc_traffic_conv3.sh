#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the features.3 backward conv (per-clone and clone-sharing kernels).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
for cl in 0 1; do
  for c in FETCH_SIZE WRITE_SIZE; do
    DRSA_AMD_CONV_CLONES=$cl timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $c --output-format csv \
      -d $O/cl${cl}_$c -o run -- python scripts/run_conv_bwd3.py > $O/cl${cl}_$c.log 2>&1
  done
done
