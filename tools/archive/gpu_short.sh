# Cold-box short headline runs (the driver's steps 20 / warmup 5) with batch traces.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --json-out gpurun_out/short_$i.json \
    --trace-out gpurun_out/short_trace_$i.json > gpurun_out/short_$i.log 2>&1 || exit 1
done
