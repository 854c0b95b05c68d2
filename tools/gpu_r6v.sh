#!/bin/bash
# Round 6: Llama-3-8B TP=1 serving on the native engine loop, 1 vs 2 compute streams (TP = 1 has no collectives).
set -o pipefail
O=gpurun_out/r6v
mkdir -p $O
export PYTHONUNBUFFERED=1
for rep in 1 2; do
  timeout -k 10 400 python bench/llama_tp_bench.py --serve --loop native --requests 400 --concurrency 16 \
      --json-out $O/cs1_$rep.json > $O/cs1_$rep.log 2>&1 || { tail -20 $O/cs1_$rep.log; exit 1; }
  timeout -k 10 400 python bench/llama_tp_bench.py --serve --loop native --requests 400 --concurrency 24 --compute-streams 2 \
      --pipeline-depth 3 --json-out $O/cs2_$rep.json > $O/cs2_$rep.log 2>&1 || { tail -20 $O/cs2_$rep.log; exit 1; }
done
python - <<'PY'
import json
for n in ["cs1_1","cs2_1","cs1_2","cs2_2"]:
    d=json.load(open(f"gpurun_out/r6v/{n}.json")); print(n, d["prompts_per_s"], d["p50_ms"], d["p99_ms"], d["mean_batch"])
PY
