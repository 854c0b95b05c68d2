#!/bin/bash
# Round 6: Poisson tails of the BERT headline engine, SDMA input copy (default) vs the gather kernel
# (RDB_ENGINE_DMA_GATHER=0), interleaved x2 at 32k and 34k req/s offered (bench.py --rate, 300 steps).
set -o pipefail
O=gpurun_out/r6am
mkdir -p $O
export PYTHONUNBUFFERED=1
for rep in 1 2; do
  for r in 32000 34000; do
    for arm in dma gather; do
      if [ $arm = gather ]; then export RDB_ENGINE_DMA_GATHER=0; else unset RDB_ENGINE_DMA_GATHER; fi
      timeout -k 10 300 python bench.py --steps 600 --warmup 30 --rate $r > $O/${arm}_${r}_$rep.log 2>&1 || { tail -20 $O/${arm}_${r}_$rep.log; exit 1; }
      echo "$arm $r $rep $(grep '^{"metric"' $O/${arm}_${r}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_ms"], d["p99_ms"], d["mean_batch"])')"
    done
  done
done
