# first-layer forward ring pass unroll sweep (micro-benchmark, interleaved); NODEN=1: no den at all
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/cfring3
mkdir -p $O
for r in 1 2; do
  for n in base cfr8 cfr16; do
    L=drsa_audio_amd/lib/libdrsa_amd.so; [ $n != base ] && L=drsa_audio_amd/lib/exp/$n.so
    DRSA_AMD_LIB=$L timeout -k 10 60 python scripts/bench_first_fwd.py >> $O/micro.txt
  done
  NODEN=1 timeout -k 10 60 python scripts/bench_first_fwd.py >> $O/micro.txt
done
cat $O/micro.txt
