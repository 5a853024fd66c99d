# 4 x 8 small-map tiles: parity tests, then the headline and VGGish A/B against a library without them
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/small
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_lrp_gpu.py tests/test_engine_gpu.py \
  tests/test_vggish_gpu.py tests/test_bf16_gpu.py tests/test_bf16_bwd_gpu.py tests/test_pins_gpu.py > gpurun_out/small/t.log 2>&1
tail -1 gpurun_out/small/t.log
bash scripts/ab_bench.sh small nosmall
for r in 1 2; do
  timeout -k 10 100 python scripts/ab_vggish.py > gpurun_out/small/vgg_base_$r.json
  DRSA_AMD_LIB=drsa_audio_amd/lib/exp/nosmall.so timeout -k 10 100 python scripts/ab_vggish.py > gpurun_out/small/vgg_nosmall_$r.json
done
