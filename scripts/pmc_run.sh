#!/bin/bash
# PMC passes (separate runs, kernel-trace only) over a short bench; outputs under gpurun_out/pmc_*.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-drsa"
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
            "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  tag=$(echo $pass | cut -d' ' -f1)
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d gpurun_out/pmc_$tag -o run -- $B > gpurun_out/pmc_$tag.log 2>&1 || echo "pass $tag failed"
done
