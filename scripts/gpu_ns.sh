#!/bin/bash
# Newton-Schulz stop-rule variants: DRSA timings (base + lib/exp variants), then the DRSA parity
# tests on the first variant.  Usage: gpu_ns.sh <tag> <variant>...
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift
mkdir -p $O
timeout -k 10 300 python scripts/bench_drsa.py 200 > $O/base.json 2> $O/base.err
for n in "$@"; do
  DRSA_AMD_LIB=drsa_audio_amd/lib/exp/$n.so timeout -k 10 300 python scripts/bench_drsa.py 200 > $O/$n.json 2> $O/$n.err
done
for f in $O/*.json; do python - "$f" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[1], round(d["drsa_c3"]["ms_per_step"], 5), round(d["drsa_joint_c5"]["ms_per_joint_step"], 5),
      d["ns_iters_c3"], d["ns_iters_d128"], d["ns_iters_d100"])
PY
done
for n in "$@"; do
  DRSA_AMD_LIB=drsa_audio_amd/lib/exp/$n.so timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_drsa_gpu.py tests/test_drsa_long_gpu.py tests/test_subrel.py tests/test_grid_gpu.py > $O/pytest_$n.log 2>&1 || true
  echo "$n: $(tail -1 $O/pytest_$n.log)"
  DRSA_AMD_LIB=drsa_audio_amd/lib/exp/$n.so timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$n.log 2>&1 && echo "$n smoke ok" || echo "$n smoke FAILED"
done
