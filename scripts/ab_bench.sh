#!/bin/bash
# In-step A/B of variant libraries on the headline bench (per-kernel HIP-event times), interleaved twice.
# Usage: ab_bench.sh <tag> <name>...
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift
mkdir -p $O
for r in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --legs none --steps 20 > $O/base_$r.json 2> /dev/null
  for n in "$@"; do DRSA_AMD_LIB=drsa_audio_amd/lib/exp/$n.so timeout -k 10 200 python bench.py --no-cpu-baseline --legs none --steps 20 > $O/${n}_$r.json 2> /dev/null; done
done
