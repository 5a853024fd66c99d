# GTZAN 128-channel forwards at W >= 32 (conv_fwd:features.6) on 8 x 16 / 8 x 32 tiles vs 8 x 8: in-step A/B
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lrp_gpu.py > gpurun_out/fw_t.log 2>&1 || true
DRSA_AMD_LIB=drsa_audio_amd/lib/exp/fw16.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lrp_gpu.py > gpurun_out/fw_t16.log 2>&1
tail -1 gpurun_out/fw_t16.log
bash scripts/ab_bench.sh fwab fw16 fw32
