#!/bin/bash
# Round 6 final tree: engine stream stagger (RDB_ENGINE_STAGGER_US, opt-in) on the 3-stream BERT engine,
# driver-shaped runs interleaved x4 per arm (0 = default, 300 us, 600 us).
set -o pipefail
O=gpurun_out/r6an
mkdir -p $O
export PYTHONUNBUFFERED=1
for rep in 1 2 3 4; do
  for st in 0 300 600; do
    if [ $st = 0 ]; then unset RDB_ENGINE_STAGGER_US; else export RDB_ENGINE_STAGGER_US=$st; fi
    timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/st${st}_$rep.log 2>&1 || { tail -20 $O/st${st}_$rep.log; exit 1; }
    echo "$st $rep $(grep '^{"metric"' $O/st${st}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_ms"], d["p99_ms"])')"
  done
done
