#!/bin/bash
# Round 6: the tuner timed from replayed hipGraphs (RDB_TUNE_GRAPH, default on): GPU op tests, then fresh
# BERT / ResNet-50 tunings in context and interleaved replays against the shipped cs3 tables.
set -o pipefail
O=gpurun_out/r6s
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ops_gpu.py tests/test_models_gpu.py \
    > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
RDB_TUNE_FILE=$PWD/$O/bert_g.json timeout -k 10 500 python bench.py --steps 300 --warmup 30 --json-out $O/bert_tune.json > $O/bert_tune.log 2>&1 || { tail -20 $O/bert_tune.log; exit 1; }
RDB_TUNE_FILE=$PWD/$O/resnet_g.json timeout -k 10 500 python bench/serve_bench.py --model resnet50 --closed 96 --seconds 5 \
    --json-out $O/resnet_tune.json > $O/resnet_tune.log 2>&1 || { tail -20 $O/resnet_tune.log; exit 1; }
for rep in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 300 --warmup 30 --json-out $O/bert_ship_$rep.json > $O/bert_ship_$rep.log 2>&1 || exit 1
  RDB_TUNE_FILE=$PWD/$O/bert_g.json timeout -k 10 300 python bench.py --steps 300 --warmup 30 --json-out $O/bert_g_$rep.json > $O/bert_g_$rep.log 2>&1 || exit 1
  timeout -k 10 300 python bench/serve_bench.py --model resnet50 --closed 96 --seconds 5 --json-out $O/rn_ship_$rep.json > $O/rn_ship_$rep.log 2>&1 || exit 1
  RDB_TUNE_FILE=$PWD/$O/resnet_g.json timeout -k 10 300 python bench/serve_bench.py --model resnet50 --closed 96 --seconds 5 \
      --json-out $O/rn_g_$rep.json > $O/rn_g_$rep.log 2>&1 || exit 1
done
python - <<'PY'
import json
O="gpurun_out/r6s/"
for n in ["bert_tune"]+[f"bert_{x}_{r}" for r in (1,2,3) for x in ("ship","g")]:
    d=json.load(open(O+n+".json")); print(n, d["value"], d.get("p50_ms"), d.get("p99_ms"))
for n in ["resnet_tune"]+[f"rn_{x}_{r}" for r in (1,2,3) for x in ("ship","g")]:
    p=json.load(open(O+n+".json"))["points"][0]; print(n, p["req_per_s"], p["p50_ms"], p["p99_ms"])
PY
