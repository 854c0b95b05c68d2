# Throughput vs p99 (Poisson open loop per GPU) with the round-2 kernels and shipped tile table.
set -o pipefail
mkdir -p gpurun_out/curve2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 5000 10000 15000 20000 25000 28000 30000; do
  timeout -k 10 150 python -u bench.py --rate $r --steps 300 --warmup 30 --json-out gpurun_out/curve2/rate_$r.json > gpurun_out/curve2/rate_$r.log 2>&1 || exit 1
done
timeout -k 10 150 python -u bench.py --json-out gpurun_out/curve2/closed.json > gpurun_out/curve2/closed.log 2>&1
