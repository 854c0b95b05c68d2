# round 4: the start-up tuner with CU-time candidates in context (no shipped table): which o-projection tile it
# picks and the throughput, against the shipped table on the same box
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r4aa
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 env RDB_TUNE_FILE=gpurun_out/r4aa/tuned_fresh.json python -u bench.py --steps 2000 --warmup 50 --tile-table none \
  > gpurun_out/r4aa/bench_fresh_tune.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 2000 --warmup 50 > gpurun_out/r4aa/bench_shipped.log 2>&1
