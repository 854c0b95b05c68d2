#!/bin/bash
# Round 6: ResNet-50 with more engine streams (the shipped cs3 table replayed for all), interleaved x2.
set -o pipefail
O=gpurun_out/r6x
mkdir -p $O
export PYTHONUNBUFFERED=1
T=$PWD/ray_dynamic_batching_amd/ops/tuned/mi355x_resnet50_B32_cs3_d6.json
run() {  # name streams depth concurrency
  RDB_TUNE_FILE=$T timeout -k 10 300 python bench/serve_bench.py --model resnet50 --closed $4 --seconds 5 --compute-streams $2 \
      --pipeline-depth $3 --json-out $O/$1.json > $O/$1.log 2>&1
}
for rep in 1 2; do
  run cs3_c96_$rep 3 6 96 || exit 1
  run cs4_c128_$rep 4 8 128 || exit 1
  run cs4_c96_$rep 4 8 96 || exit 1
  run cs3_c128_$rep 3 6 128 || exit 1
done
python - <<'PY'
import json
O="gpurun_out/r6x/"
for r in (1,2):
    for n in ("cs3_c96","cs4_c128","cs4_c96","cs3_c128"):
        p=json.load(open(O+f"{n}_{r}.json"))["points"][0]; print(n, r, p["req_per_s"], p["p50_ms"], p["p99_ms"])
PY
