# first-layer forward ring pass spread over all lanes: parity, micro-benchmark, in-step A/B
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/cfringx
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_first_gpu.py \
  tests/test_conv_den_ring_gpu.py tests/test_lrp_gpu.py > $O/t.log 2>&1
tail -1 $O/t.log
for r in 1 2; do
  for n in base rx0; do
    L=drsa_audio_amd/lib/libdrsa_amd.so; [ $n != base ] && L=drsa_audio_amd/lib/exp/$n.so
    DRSA_AMD_LIB=$L timeout -k 10 60 python scripts/bench_first_fwd.py >> $O/micro.txt
  done
done
cat $O/micro.txt
bash scripts/ab_bench.sh cfringx/ab rx0
