#!/bin/bash
# Round 6 final tree: the headline metric as a curve -- BERT-base dyn-batch <= 32 req/s vs p99 on one MI355X,
# Poisson open loop at fixed offered rates (bench.py --rate, 600 steps) and the closed loop 96.
set -o pipefail
O=gpurun_out/r6al2
mkdir -p $O
export PYTHONUNBUFFERED=1
for r in 10000 20000 28000 32000 34000 35000 36000; do
  timeout -k 10 300 python bench.py --steps 600 --warmup 30 --rate $r > $O/poisson_$r.log 2>&1 || { tail -20 $O/poisson_$r.log; exit 1; }
  echo "$r $(grep '^{"metric"' $O/poisson_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_ms"], d["p99_ms"], d["mean_batch"])')"
done
