#!/bin/bash
# Micro-benchmark one script under several variant libraries, alternating, two passes.
# Usage: gpu_libs.sh <tag> <script.py> <lib names (lib/exp/<name>.so; "default" = the in-tree lib)...>
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; S=$2; shift 2
mkdir -p $O
for pass in 1 2; do
  for n in "$@"; do
    if [ "$n" = default ]; then L=; else L=DRSA_AMD_LIB=drsa_audio_amd/lib/exp/$n.so; fi
    env $L timeout -k 10 120 python $S >> $O/libs.jsonl 2>> $O/libs.err
  done
done
cat $O/libs.jsonl
