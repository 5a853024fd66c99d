# projection_bwd micro-benchmark: default library vs the variants named on the command line
set -e
mkdir -p gpurun_out/pb
O=gpurun_out/pb/pb.log
: > $O
timeout -k 10 60 python scripts/bench_projection_bwd.py >> $O 2>&1
for v in "$@"; do DRSA_AMD_LIB=drsa_audio_amd/lib/exp/$v.so timeout -k 10 60 python scripts/bench_projection_bwd.py >> $O 2>&1; done
