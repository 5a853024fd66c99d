#!/bin/bash
# SQ counter passes for the three kernels after the dominant one: first-layer backward, conv3 backward, projection backward
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
bash scripts/pmc_kernel.sh gpurun_out/pmc_fl first_layer_bwd_pooled scripts/bench_first_layer.py
bash scripts/pmc_kernel.sh gpurun_out/pmc_c3 conv3x3 scripts/run_conv_bwd3.py
bash scripts/pmc_kernel.sh gpurun_out/pmc_pb projection_bwd scripts/bench_projection_bwd.py
