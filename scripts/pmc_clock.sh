#!/bin/bash
# Effective clock and MFMA-pipe occupancy of one kernel (how far the conv
# backward sits from the fp32 MFMA rate the chip sustains):
#   clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel wall time; MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES /
#   (GRBM_GUI_ACTIVE / 8 * 256 CUs * 4 SIMDs)
#   pmc_clock.sh <out_dir> <kernel_regex> <python script ...>
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$1; RX=$2; shift 2
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVE_CYCLES \
  --kernel-include-regex "$RX" --output-format csv -d $OUT/clk -o run -- python "$@" > $OUT/clk.log 2>&1
