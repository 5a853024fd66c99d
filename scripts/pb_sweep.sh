set -e
mkdir -p gpurun_out/pb
O=gpurun_out/pb/pb.log
: > $O
RC=0 timeout -k 10 60 python scripts/bench_projection_bwd.py >> $O 2>&1
timeout -k 10 60 python scripts/bench_projection_bwd.py >> $O 2>&1
for v in rcw1 rcpt1 rcpt8; do DRSA_AMD_LIB=drsa_audio_amd/lib/exp/$v.so timeout -k 10 60 python scripts/bench_projection_bwd.py >> $O 2>&1; done
