set -eo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$1
for v in base pold pw4 base pold pw4; do
  L=drsa_audio_amd/lib/libdrsa_amd.so; [ $v != base ] && L=drsa_audio_amd/lib/exp/$v.so
  echo -n "$v proj " >> gpurun_out/$1/proj.txt
  DRSA_AMD_LIB=$L timeout -k 10 120 python scripts/bench_projection_bwd.py >> gpurun_out/$1/proj.txt
done
cat gpurun_out/$1/proj.txt
