#!/bin/bash
# A/B of an env switch on the bench: ab_env.sh <tag> <VAR> <val1> <val2> ...
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; VAR=$2; shift 2
mkdir -p $O
for v in "$@"; do
  env $VAR=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-drsa > $O/bench_$v.json 2> $O/bench_$v.err
done
