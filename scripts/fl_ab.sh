set -eo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4d
for v in flold fld1 fld2 fld3 flold fld1 fld2 fld3; do
  echo -n "$v " >> gpurun_out/r4d/fl.txt
  DRSA_AMD_LIB=drsa_audio_amd/lib/exp/$v.so timeout -k 10 120 python scripts/bench_first_layer.py >> gpurun_out/r4d/fl.txt
done
