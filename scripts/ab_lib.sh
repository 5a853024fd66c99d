#!/bin/bash
# A/B of variant libraries (lib/exp/<name>.so) on one micro-bench script, interleaved twice.
# Usage: ab_lib.sh <tag> <bench script> <name>...
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; S=$2; shift 2
mkdir -p $O
for r in 1 2; do
  timeout -k 10 100 python $S > $O/base_$r.json
  for n in "$@"; do DRSA_AMD_LIB=drsa_audio_amd/lib/exp/$n.so timeout -k 10 100 python $S > $O/${n}_$r.json; done
done
for f in $O/*.json; do echo "$f $(python -c "import json,sys; d=json.load(open('$f')); print(d.get('ms_per_launch', d.get('ms')))")"; done
