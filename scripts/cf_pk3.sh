set -eo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/cfpk3
mkdir -p $O
for r in 1 2; do
  timeout -k 10 60 python scripts/bench_first_fwd.py >> $O/micro.txt
  NODEN=1 timeout -k 10 60 python scripts/bench_first_fwd.py >> $O/micro.txt
  RING=0 timeout -k 10 60 python scripts/bench_first_fwd.py >> $O/micro.txt
done
cat $O/micro.txt
