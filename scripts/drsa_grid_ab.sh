set -eo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$1
for gsz in 0 128 64 32 0 128 64 32; do
  echo -n "grid=$gsz " >> gpurun_out/$1/dg.txt
  DRSA_AMD_PARTIAL_GRID=$gsz timeout -k 10 200 python scripts/bench_drsa.py 200 2>/dev/null | tr -d '\n' | cut -c1-400 >> gpurun_out/$1/dg.txt
  echo >> gpurun_out/$1/dg.txt
done
cat gpurun_out/$1/dg.txt
