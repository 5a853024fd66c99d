# first-layer forward occupancy / unroll sweep (micro-benchmark, interleaved)
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/cfpk2
mkdir -p $O
for r in 1 2; do
  for n in base cfold cfw5 cfu2 cfu1w6; do
    L=drsa_audio_amd/lib/libdrsa_amd.so; [ $n != base ] && L=drsa_audio_amd/lib/exp/$n.so
    DRSA_AMD_LIB=$L timeout -k 10 60 python scripts/bench_first_fwd.py >> $O/micro.txt
  done
done
cat $O/micro.txt
