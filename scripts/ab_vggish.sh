# VGGish fp32 standard-LRP A/B: the main library against variant libraries under drsa_audio_amd/lib/exp
#   bash scripts/ab_vggish.sh <variant> [<variant> ...]
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/vab
for r in 1 2; do
  timeout -k 10 100 python scripts/ab_vggish.py > gpurun_out/vab/base_$r.json
  for n in "$@"; do DRSA_AMD_LIB=drsa_audio_amd/lib/exp/$n.so timeout -k 10 100 python scripts/ab_vggish.py > gpurun_out/vab/${n}_$r.json; done
done
