#!/bin/bash
# rocprofv3 kernel-trace stats of one bench.py run + per-tag timing.  Usage: prof_bench.sh <tag> [bench args]
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p $O
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python bench.py --tag-order $O/prof_tags.json "$@" > $O/prof_bench.json 2> $O/prof_bench.err
python scripts/tag_profile.py trace $O/prof $O/prof_tags.json $O/prof_tags_timing.json > /dev/null
