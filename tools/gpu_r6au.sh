#!/bin/bash
# Round 6 closing: three more fresh in-context cs3 tunings of the ResNet-50 serving engine vs the re-tuned shipped table (the
# halo tiles got faster, so the tuner may now pick them for more layers) vs the shipped cs3 table, closed loop 128,
# interleaved x2.
set -o pipefail
O=gpurun_out/r6au
mkdir -p $O
export PYTHONUNBUFFERED=1
S=$PWD/ray_dynamic_batching_amd/ops/tuned/mi355x_resnet50_B32_cs3_d6.json
for t in 1 2 3; do
  rm -f $O/t$t.json
  RDB_TUNE_FILE=$PWD/$O/t$t.json timeout -k 10 500 python bench/serve_bench.py --model resnet50 --closed 128 --seconds 3 \
      --json-out $O/tune_$t.json > $O/tune_$t.log 2>&1 || { tail -20 $O/tune_$t.log; exit 1; }
  [ -s $O/t$t.json ] || { echo "no table"; exit 1; }
done
for rep in 1 2; do
  for t in s 1 2 3; do
    f=$S; [ $t = s ] || f=$PWD/$O/t$t.json
    RDB_TUNE_FILE=$f timeout -k 10 300 python bench/serve_bench.py --model resnet50 --closed 128 --seconds 5 \
        --json-out $O/run_${t}_$rep.json > $O/run_${t}_$rep.log 2>&1 || { tail -20 $O/run_${t}_$rep.log; exit 1; }
    python3 -c "import json; p=json.load(open('$O/run_${t}_$rep.json'))['points'][0]; print('$t $rep', p['req_per_s'], p['p50_ms'], p['p99_ms'])"
  done
done
