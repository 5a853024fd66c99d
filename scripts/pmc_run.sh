#!/bin/bash
# HBM traffic passes for the bench workload: FETCH_SIZE and WRITE_SIZE in separate rocprofv3 runs
# (kernel-trace only, no other tracing), mapped to engine tags by scripts/tag_profile.py.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc}
mkdir -p $OUT
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $OUT/pmc_$c -o run -- \
    python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-drsa --tag-order $OUT/tags_$c.json \
    > $OUT/pmc_$c.log 2>&1
done
cp $OUT/tags_FETCH_SIZE.json $OUT/tags.json
python scripts/tag_profile.py pmc $OUT $OUT/tags.json $OUT/pmc_traffic.json > /dev/null
