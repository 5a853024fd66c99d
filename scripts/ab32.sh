set -eo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$1
for v in base old base old; do
  L=drsa_audio_amd/lib/libdrsa_amd.so; [ $v != base ] && L=drsa_audio_amd/lib/exp/$v.so
  echo -n "$v proj " >> gpurun_out/$1/ab.txt; DRSA_AMD_LIB=$L timeout -k 10 120 python scripts/bench_projection_bwd.py >> gpurun_out/$1/ab.txt
  echo -n "$v flpool " >> gpurun_out/$1/ab.txt; DRSA_AMD_LIB=$L timeout -k 10 120 python scripts/bench_first_layer.py >> gpurun_out/$1/ab.txt
  echo -n "$v fldense " >> gpurun_out/$1/ab.txt; FL_DENSE=1 DRSA_AMD_LIB=$L timeout -k 10 120 python scripts/bench_first_layer.py >> gpurun_out/$1/ab.txt
done
cat gpurun_out/$1/ab.txt
