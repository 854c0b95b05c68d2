# Five driver-shaped short headline runs (steps 20 / warmup 5) with batch traces, fresh processes.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for i in 1 2 3 4 5; do
  timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --json-out gpurun_out/s5_$i.json \
    --trace-out gpurun_out/s5_trace_$i.json > gpurun_out/s5_$i.log 2>&1 || exit 1
done
