#!/bin/bash
# Round 6: shipped ResNet table vs the same table with stage 2's bs32 3x3 on halo tile 5 (graph-timed x3 13.0 vs 16.1 us).
set -o pipefail
O=gpurun_out/r6u
mkdir -p $O
export PYTHONUNBUFFERED=1
for rep in 1 2 3; do
  timeout -k 10 300 python bench/serve_bench.py --model resnet50 --closed 96 --seconds 5 --json-out $O/b_$rep.json > $O/b_$rep.log 2>&1 || exit 1
  RDB_TUNE_FILE=$PWD/bench/tables_tmp/resnet_b_s2h5.json timeout -k 10 300 python bench/serve_bench.py --model resnet50 --closed 96 \
      --seconds 5 --json-out $O/h5_$rep.json > $O/h5_$rep.log 2>&1 || exit 1
done
python - <<'PY'
import json
O="gpurun_out/r6u/"
for n in [f"{x}_{r}" for r in (1,2,3) for x in ("b","h5")]:
    p=json.load(open(O+n+".json"))["points"][0]; print(n, p["req_per_s"], p["p50_ms"], p["p99_ms"])
PY
