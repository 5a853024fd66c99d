set -eo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$1
for v in base cc4 cc2 base cc4 cc2; do
  L=drsa_audio_amd/lib/libdrsa_amd.so; [ $v != base ] && L=drsa_audio_amd/lib/exp/$v.so
  echo -n "$v " >> gpurun_out/$1/fl.txt
  FL_DENSE=1 DRSA_AMD_LIB=$L timeout -k 10 120 python scripts/bench_first_layer.py >> gpurun_out/$1/fl.txt
done
cat gpurun_out/$1/fl.txt
