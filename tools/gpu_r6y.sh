#!/bin/bash
# Round 6: ResNet-50 (3 x 6 engine, shipped table) capacity: closed loops 128 / 160 / 192 in flight and Poisson
# offered rates around it; BERT closed 128 for the same question.
set -o pipefail
O=gpurun_out/r6y
mkdir -p $O
export PYTHONUNBUFFERED=1
for c in 128 160 192; do
  timeout -k 10 300 python bench/serve_bench.py --model resnet50 --closed $c --seconds 5 --json-out $O/rn_c$c.json > $O/rn_c$c.log 2>&1 || exit 1
done
timeout -k 10 600 python bench/serve_bench.py --model resnet50 --rates 44000,46000,48000,50000 --seconds 4 \
    --json-out $O/rn_poisson.json > $O/rn_poisson.log 2>&1 || exit 1
timeout -k 10 300 python bench/serve_bench.py --model resnet50 --closed 128 --seconds 5 --json-out $O/rn_c128b.json > $O/rn_c128b.log 2>&1 || exit 1
python - <<'PY'
import json
O="gpurun_out/r6y/"
for n in ("rn_c128","rn_c160","rn_c192","rn_c128b"):
    p=json.load(open(O+n+".json"))["points"][0]; print(n, p["req_per_s"], p["p50_ms"], p["p99_ms"], p["mean_batch"])
for p in json.load(open(O+"rn_poisson.json"))["points"]: print("poisson", p["offered"], p["req_per_s"], p["p50_ms"], p["p99_ms"], p["mean_batch"])
PY
