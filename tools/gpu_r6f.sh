#!/bin/bash
# Round 6: the 3-stream default on the driver's command (x10), two more cs3 BERT tunings vs the
# shipped cs3 table, and ResNet-50 at 2 x 4 (shipped table) vs 3 x 6 (tuned here, saved).
set -o pipefail
O=gpurun_out/r6f
mkdir -p $O
export PYTHONUNBUFFERED=1
for i in 1 2 3 4 5 6 7 8 9 10; do
  timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out $O/bench_$i.json > $O/bench_$i.log 2>&1 || exit 1
done
for t in a b; do
  RDB_TUNE_FILE=$PWD/$O/table_cs3_$t.json timeout -k 10 300 python bench.py --steps 300 --warmup 30 \
      --json-out $O/tune_cs3_$t.json > $O/tune_cs3_$t.log 2>&1 || exit 1
  RDB_TUNE_FILE=$PWD/$O/table_cs3_$t.json timeout -k 10 300 python bench.py --steps 300 --warmup 30 \
      --json-out $O/replay_cs3_$t.json > $O/replay_cs3_$t.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --steps 300 --warmup 30 --json-out $O/shipped_cs3_$t.json > $O/shipped_cs3_$t.log 2>&1 || exit 1
done
for rep in 1 2; do
  timeout -k 10 300 python bench/serve_bench.py --model resnet50 --closed 96 --seconds 5 \
      --json-out $O/resnet_cs2_$rep.json > $O/resnet_cs2_$rep.log 2>&1 || exit 1
  RDB_TUNE_FILE=$PWD/$O/table_resnet_cs3_d6.json timeout -k 10 400 python bench/serve_bench.py --model resnet50 \
      --closed 96 --seconds 5 --compute-streams 3 --pipeline-depth 6 \
      --json-out $O/resnet_cs3_$rep.json > $O/resnet_cs3_$rep.log 2>&1 || exit 1
done
echo "exit 0"
