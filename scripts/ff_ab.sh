set -eo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$1
for v in base ffnodpp base ffnodpp; do
  L=drsa_audio_amd/lib/libdrsa_amd.so; [ $v != base ] && L=drsa_audio_amd/lib/exp/$v.so
  DRSA_AMD_LIB=$L timeout -k 10 120 python scripts/bench_fused_first.py >> gpurun_out/$1/ff.txt
done
DRSA_AMD_FF_DBG=1 timeout -k 10 120 python scripts/bench_fused_first.py >> gpurun_out/$1/ff.txt
DRSA_AMD_FF_DBG=2 timeout -k 10 120 python scripts/bench_fused_first.py >> gpurun_out/$1/ff.txt
cat gpurun_out/$1/ff.txt
