set -eo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$1
for v in base pt1 pt2 wpe4 wpe2 plds base; do
  L=drsa_audio_amd/lib/libdrsa_amd.so; [ $v != base ] && [ $v != plds ] && L=drsa_audio_amd/lib/exp/$v.so
  P=0; [ $v == plds ] && P=1
  echo -n "$v proj " >> gpurun_out/$1/proj.txt
  DRSA_AMD_PROJ_PLDS=$P DRSA_AMD_LIB=$L timeout -k 10 120 python scripts/bench_projection_bwd.py >> gpurun_out/$1/proj.txt
done
cat gpurun_out/$1/proj.txt
