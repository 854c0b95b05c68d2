#!/bin/bash
# Round 6 closing: two fresh in-context cs3 tunings of the BERT dyn-batch <= 16 engine (config 3) vs the shipped
# against the shipped cs3 table, interleaved x2 (300 steps): ship a new table only if it wins every pair.
set -o pipefail
O=gpurun_out/r6at
mkdir -p $O
export PYTHONUNBUFFERED=1
B="python bench.py --steps 300 --warmup 30 --max-batch 16"
S=$PWD/ray_dynamic_batching_amd/ops/tuned/mi355x_bert_L12_S128_B16_cs3_d6.json
for t in 1 2; do
  rm -f $O/t$t.json
  RDB_TUNE_FILE=$PWD/$O/t$t.json timeout -k 10 400 $B > $O/tune_$t.log 2>&1 || { tail -20 $O/tune_$t.log; exit 1; }
  [ -s $O/t$t.json ] || { echo "no table written"; exit 1; }
done
for rep in 1 2; do
  for t in s 1 2; do
    f=$S; [ $t = s ] || f=$PWD/$O/t$t.json
    RDB_TUNE_FILE=$f timeout -k 10 300 $B > $O/run_${t}_$rep.log 2>&1 || { tail -20 $O/run_${t}_$rep.log; exit 1; }
    echo "$t $rep $(grep '^{"metric"' $O/run_${t}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_ms"], d["p99_ms"])')"
  done
done
