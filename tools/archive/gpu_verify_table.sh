# Headline with the shipped tile table: 4 driver-shaped short runs, then one default run.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for i in 1 2 3 4; do
  timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --json-out gpurun_out/vt_s_$i.json > gpurun_out/vt_s_$i.log 2>&1 || exit 1
done
timeout -k 10 200 python -u bench.py --json-out gpurun_out/vt_long.json > gpurun_out/vt_long.log 2>&1
