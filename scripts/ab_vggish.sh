set -eo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/vab
timeout -k 10 600 python -u -m pytest tests/test_vggish_gpu.py tests/test_pool24_fp32_gpu.py tests/test_bf16_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/vab/pytest.log 2>&1
for r in 1 2; do
  timeout -k 10 100 python scripts/ab_vggish.py > gpurun_out/vab/base_$r.json
  for n in f128t8 f128t16; do DRSA_AMD_LIB=drsa_audio_amd/lib/exp/$n.so timeout -k 10 100 python scripts/ab_vggish.py > gpurun_out/vab/${n}_$r.json; done
done
