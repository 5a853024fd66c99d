#!/bin/bash
# log-mel tests + micro-bench + per-phase cycle profile (lib/exp/lfprof.so).  Usage: gpu_lmp.sh <tag>
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_logmel_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
timeout -k 10 120 python scripts/bench_frontend.py > $O/b.json 2> $O/b.err
DRSA_AMD_LIB=drsa_audio_amd/lib/exp/lfprof.so timeout -k 10 120 python scripts/logmel_phases.py > $O/phases.json
for n in head; do DRSA_AMD_LIB=drsa_audio_amd/lib/exp/$n.so timeout -k 10 120 python scripts/bench_frontend.py > $O/$n.json; done
tail -2 $O/t.log; for f in b head; do echo $f; cat $O/$f.json; done; cat $O/phases.json
