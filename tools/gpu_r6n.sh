#!/bin/bash
# Round 6: confirm the halo ResNet table (a second fresh tuning b, then shipped / a / b interleaved x3).
set -o pipefail
O=gpurun_out/r6n
mkdir -p $O
export PYTHONUNBUFFERED=1
RDB_TUNE_FILE=$PWD/$O/table_halo_b.json timeout -k 10 400 python bench/serve_bench.py --model resnet50 --closed 96 --seconds 5 \
    --json-out $O/tune_halo_b.json > $O/tune_halo_b.log 2>&1 || { tail -20 $O/tune_halo_b.log; exit 1; }
for rep in 1 2 3; do
  timeout -k 10 300 python bench/serve_bench.py --model resnet50 --closed 96 --seconds 5 \
      --json-out $O/ship_$rep.json > $O/ship_$rep.log 2>&1 || exit 1
  RDB_TUNE_FILE=$PWD/bench/tables_tmp/resnet_halo_a.json timeout -k 10 300 python bench/serve_bench.py --model resnet50 --closed 96 \
      --seconds 5 --json-out $O/a_$rep.json > $O/a_$rep.log 2>&1 || exit 1
  RDB_TUNE_FILE=$PWD/$O/table_halo_b.json timeout -k 10 300 python bench/serve_bench.py --model resnet50 --closed 96 \
      --seconds 5 --json-out $O/b_$rep.json > $O/b_$rep.log 2>&1 || exit 1
done
python - <<'PY'
import json
O="gpurun_out/r6n/"
for n in ["tune_halo_b"]+[f"{x}_{r}" for r in (1,2,3) for x in ("ship","a","b")]:
    p=json.load(open(O+n+".json"))["points"][0]; print(n, p["req_per_s"], p["p50_ms"], p["p99_ms"])
PY
