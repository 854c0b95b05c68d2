#!/bin/bash
# Round 6: serving curves on the final defaults (3 streams x depth 6, shipped cs3 tables):
# BERT (bench.py Poisson rates + closed loop, timeout policy) and ResNet-50 (serve_bench Poisson + closed).
set -o pipefail
O=gpurun_out/r6p
mkdir -p $O
export PYTHONUNBUFFERED=1
for r in 5000 10000 20000 28000 34000; do
  timeout -k 10 300 python bench.py --rate $r --steps 200 --warmup 20 --json-out $O/bert_r$r.json > $O/bert_r$r.log 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --steps 300 --warmup 30 --json-out $O/bert_closed.json > $O/bert_closed.log 2>&1 || exit 1
timeout -k 10 600 python bench/serve_bench.py --model resnet50 --rates 8000,16000,24000,32000,40000 --closed 96 --seconds 4 \
    --json-out $O/resnet_curve.json > $O/resnet_curve.log 2>&1 || exit 1
python - <<'PY'
import json
O="gpurun_out/r6p/"
for r in (5000,10000,20000,28000,34000):
    d=json.load(open(O+f"bert_r{r}.json")); print("bert", r, d["value"], d.get("p50_ms"), d.get("p99_ms"))
d=json.load(open(O+"bert_closed.json")); print("bert closed", d["value"], d.get("p50_ms"), d.get("p99_ms"))
for p in json.load(open(O+"resnet_curve.json"))["points"]: print("resnet", p["load"], p["offered"], p["req_per_s"], p["p50_ms"], p["p99_ms"], p["mean_batch"])
PY
