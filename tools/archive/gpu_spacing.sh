# Launch-spacing sweep (RDB_LAUNCH_SPACING_US) on one box with a fixed tile table, 2 rounds.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -f gpurun_out/sp_tiles.json
export RDB_TUNE_FILE=$GRAFT_REPO_ROOT/gpurun_out/sp_tiles.json
timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 > gpurun_out/sp_tune.log 2>&1 || exit 1
for r in 1 2; do
  for sp in 0 40 80 130 250; do
    timeout -k 10 200 env RDB_LAUNCH_SPACING_US=$sp python -u bench.py --steps 600 --warmup 30 \
      --json-out gpurun_out/sp_${sp}_$r.json > gpurun_out/sp_${sp}_$r.log 2>&1 || exit 1
  done
done
timeout -k 10 200 env RDB_LAUNCH_SPACING_US=80 python -u bench.py --steps 40 --warmup 5 \
  --trace-out gpurun_out/sp_trace_80.json > gpurun_out/sp_trace.log 2>&1
