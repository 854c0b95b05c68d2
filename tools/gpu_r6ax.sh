#!/bin/bash
# Round 6 closing: ResNet-50 serving under Poisson arrivals with the shipped (re-tuned) cs3 table.
set -o pipefail
O=gpurun_out/r6ax
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python bench/serve_bench.py --model resnet50 --rates 44000,48000,50000,52000 --seconds 4 \
    --json-out $O/rn_poisson.json > $O/rn_poisson.log 2>&1 || { tail -20 $O/rn_poisson.log; exit 1; }
python3 -c "
import json
for p in json.load(open('$O/rn_poisson.json'))['points']: print(p['offered'], p['req_per_s'], p['p50_ms'], p['p99_ms'], p['mean_batch'])"
