#!/bin/bash
# SQ counter passes (one rocprofv3 --pmc run per set, kernel-trace only) for one kernel regex.
#   pmc_kernel.sh <out_dir> <kernel_regex> <python script ...>
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$1; RX=$2; shift 2
mkdir -p $OUT
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --kernel-include-regex "$RX" --output-format csv \
    -d $OUT/pmc_$i -o run -- python "$@" > $OUT/pmc_$i.log 2>&1
done
python scripts/pmc_summary.py $OUT > $OUT/summary.txt 2>&1 || true
