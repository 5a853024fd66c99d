set -eo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$1
for v in base cfold cfu1 cfu2 base cfold cfu1 cfu2; do
  L=drsa_audio_amd/lib/libdrsa_amd.so; [ $v != base ] && L=drsa_audio_amd/lib/exp/$v.so
  DRSA_AMD_LIB=$L timeout -k 10 120 python scripts/bench_first_fwd.py >> gpurun_out/$1/cf.txt
done
cat gpurun_out/$1/cf.txt
