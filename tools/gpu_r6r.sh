#!/bin/bash
# Round 6: BERT dyn-batch <= 16 (BASELINE config 3) on the 3-stream engine: tune a cs3 table in context,
# replay it vs the round-3 cs2 B16 table; ResNet-50 re-tune with the split-K halo tiles (table c) vs shipped b.
set -o pipefail
O=gpurun_out/r6r
mkdir -p $O
export PYTHONUNBUFFERED=1
RDB_TUNE_FILE=$PWD/$O/bert_b16_cs3.json timeout -k 10 400 python bench.py --max-batch 16 --steps 300 --warmup 30 \
    --json-out $O/b16_tune.json > $O/b16_tune.log 2>&1 || { tail -20 $O/b16_tune.log; exit 1; }
for rep in 1 2; do
  RDB_TUNE_FILE=$PWD/$O/bert_b16_cs3.json timeout -k 10 300 python bench.py --max-batch 16 --steps 300 --warmup 30 \
      --json-out $O/b16_cs3_$rep.json > $O/b16_cs3_$rep.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --max-batch 16 --steps 300 --warmup 30 --compute-streams 2 --pipeline-depth 4 \
      --json-out $O/b16_cs2_$rep.json > $O/b16_cs2_$rep.log 2>&1 || exit 1
done
RDB_TUNE_FILE=$PWD/$O/resnet_c.json timeout -k 10 400 python bench/serve_bench.py --model resnet50 --closed 96 --seconds 5 \
    --json-out $O/resnet_tune_c.json > $O/resnet_tune_c.log 2>&1 || { tail -20 $O/resnet_tune_c.log; exit 1; }
for rep in 1 2 3; do
  timeout -k 10 300 python bench/serve_bench.py --model resnet50 --closed 96 --seconds 5 --json-out $O/rb_$rep.json > $O/rb_$rep.log 2>&1 || exit 1
  RDB_TUNE_FILE=$PWD/$O/resnet_c.json timeout -k 10 300 python bench/serve_bench.py --model resnet50 --closed 96 --seconds 5 \
      --json-out $O/rc_$rep.json > $O/rc_$rep.log 2>&1 || exit 1
done
python - <<'PY'
import json
O="gpurun_out/r6r/"
for n in ["b16_tune","b16_cs3_1","b16_cs2_1","b16_cs3_2","b16_cs2_2"]:
    d=json.load(open(O+n+".json")); print(n, d["value"], d.get("p50_ms"), d.get("p99_ms"), d["config"].get("tile_table"))
for n in ["resnet_tune_c","rb_1","rc_1","rb_2","rc_2","rb_3","rc_3"]:
    p=json.load(open(O+n+".json"))["points"][0]; print(n, p["req_per_s"], p["p50_ms"], p["p99_ms"])
PY
