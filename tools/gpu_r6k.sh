#!/bin/bash
# Round 6: ResNet-50 serving with the halo-tile 3x3 convs in the tuner's candidate set:
# halo numerics, a fresh cs3/d6 tuning (table saved), then shipped vs new table interleaved.
set -o pipefail
O=gpurun_out/r6k
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "halo" \
    > $O/pytest_halo.log 2>&1 || { tail -30 $O/pytest_halo.log; exit 1; }
tail -1 $O/pytest_halo.log
RDB_TUNE_FILE=$PWD/$O/table_halo_a.json timeout -k 10 400 python bench/serve_bench.py --model resnet50 --closed 96 --seconds 5 \
    --json-out $O/tune_halo_a.json > $O/tune_halo_a.log 2>&1 || { tail -20 $O/tune_halo_a.log; exit 1; }
for rep in 1 2; do
  timeout -k 10 300 python bench/serve_bench.py --model resnet50 --closed 96 --seconds 5 \
      --json-out $O/ship_$rep.json > $O/ship_$rep.log 2>&1 || exit 1
  RDB_TUNE_FILE=$PWD/$O/table_halo_a.json timeout -k 10 300 python bench/serve_bench.py --model resnet50 --closed 96 \
      --seconds 5 --json-out $O/halo_$rep.json > $O/halo_$rep.log 2>&1 || exit 1
done
python - <<'PY'
import json
O="gpurun_out/r6k/"
t=json.load(open(O+"table_halo_a.json"))
print("halo picks:", [(k[2],k[4],k[5],hex(c)) for k,c in t if k[0]=="conv" and c >= (1<<18)])
for n in ["tune_halo_a","ship_1","halo_1","ship_2","halo_2"]:
    p=json.load(open(O+n+".json"))["points"][0]; print(n, p["req_per_s"], p["p50_ms"], p["p99_ms"])
PY
