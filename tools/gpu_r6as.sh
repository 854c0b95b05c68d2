#!/bin/bash
# Round 6: confirmation of the re-tuned ResNet-50 cs3 table (candidate, tools/gpu_r6ar.sh t2) vs the shipped one,
# closed loop 128, interleaved x3 on a fresh box.
set -o pipefail
O=gpurun_out/${OUT:-r6as}
mkdir -p $O
export PYTHONUNBUFFERED=1
S=$PWD/ray_dynamic_batching_amd/ops/tuned/mi355x_resnet50_B32_cs3_d6.json
C=$PWD/$1
for rep in 1 2 3; do
  for t in s c; do
    f=$S; [ $t = c ] && f=$C
    RDB_TUNE_FILE=$f timeout -k 10 300 python bench/serve_bench.py --model resnet50 --closed 128 --seconds 5 \
        --json-out $O/run_${t}_$rep.json > $O/run_${t}_$rep.log 2>&1 || { tail -20 $O/run_${t}_$rep.log; exit 1; }
    python3 -c "import json; p=json.load(open('$O/run_${t}_$rep.json'))['points'][0]; print('$t $rep', p['req_per_s'], p['p50_ms'], p['p99_ms'])"
  done
done
