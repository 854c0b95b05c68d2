set -o pipefail
mkdir -p gpurun_out/curve
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 5000 10000 15000 20000 24000 26000; do
  timeout -k 10 150 python -u bench.py --rate $r --steps 300 --warmup 30 --json-out gpurun_out/curve/rate_$r.json > gpurun_out/curve/rate_$r.log 2>&1 || exit 1
done
timeout -k 10 150 python -u bench.py --json-out gpurun_out/curve/closed.json > gpurun_out/curve/closed.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o b -- python3 bench.py --steps 200 > gpurun_out/prof_bench.log 2>&1
