#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, rocprofv3 kernel-trace stats of the bench command,
# PMC HBM-traffic passes.  Every GPU step has its own time limit; the first failure ends the script.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-round}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python bench.py --tag-order $O/prof_tags.json > $O/prof_bench.json 2> $O/prof_bench.err
python scripts/tag_profile.py trace $O/prof $O/prof_tags.json $O/prof_tags_timing.json > /dev/null
bash scripts/pmc_run.sh $O/pmc
