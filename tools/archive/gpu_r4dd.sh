# round 4: ResNet-50 table tuned from scratch with the CU-time in-context candidates (conv + dense keys)
# vs the shipped table, same box, 2 rounds
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r4dd
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 1 2; do
  timeout -k 10 240 python -u bench/serve_bench.py --model resnet50 --closed 96 --seconds 5 \
    > gpurun_out/r4dd/shipped_r$r.log 2>&1 || exit $?
  timeout -k 10 400 env RDB_TUNE_STREAMS=2 RDB_TUNE_FILE=gpurun_out/r4dd/tiles_fresh_r$r.json python -u bench/serve_bench.py \
    --model resnet50 --closed 96 --seconds 5 > gpurun_out/r4dd/fresh_r$r.log 2>&1 || exit $?
  echo "r$r shipped $(tail -n 1 gpurun_out/r4dd/shipped_r$r.log) fresh $(tail -n 1 gpurun_out/r4dd/fresh_r$r.log)" >> gpurun_out/r4dd/ab.txt
done
