# first-layer forward: channels split over grid.y (2 / 4 slices) vs one slice; parity + micro-benchmark
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/cfcs
mkdir -p $O
DRSA_AMD_LIB=drsa_audio_amd/lib/exp/cs2.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_conv_first_gpu.py tests/test_conv_den_ring_gpu.py > $O/t.log 2>&1
tail -1 $O/t.log
for r in 1 2; do
  for n in base cs2 cs4; do
    L=drsa_audio_amd/lib/libdrsa_amd.so; [ $n != base ] && L=drsa_audio_amd/lib/exp/$n.so
    DRSA_AMD_LIB=$L timeout -k 10 60 python scripts/bench_first_fwd.py >> $O/micro.txt
  done
done
cat $O/micro.txt
