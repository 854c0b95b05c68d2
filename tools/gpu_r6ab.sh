#!/bin/bash
# Round 6: strided-SDMA engine input copy as the default -- engine GPU tests (incl. ring wrap on
# both paths), BERT driver-shaped runs x6 and ResNet-50 closed loop 128 x2.
set -o pipefail
O=gpurun_out/r6ab
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_models_gpu.py -k "engine" tests/test_models2_gpu.py > $O/pytest_engine.log 2>&1 || { tail -30 $O/pytest_engine.log; exit 1; }
tail -3 $O/pytest_engine.log
for i in 1 2 3 4 5 6; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bert_drv_$i.log 2>&1 || { tail -20 $O/bert_drv_$i.log; exit 1; }
done
for i in 1 2; do
  timeout -k 10 300 python bench/serve_bench.py --model resnet50 --closed 128 --seconds 5 \
      --json-out $O/rn_$i.json > $O/rn_$i.log 2>&1 || { tail -20 $O/rn_$i.log; exit 1; }
done
python - <<'PY'
import json, glob
O="gpurun_out/r6ab/"
for f in sorted(glob.glob(O+"rn_*.json")):
    p=json.load(open(f))["points"][0]; print(f.split("/")[-1], p["req_per_s"], p["p50_ms"], p["p99_ms"], p["mean_batch"])
for f in sorted(glob.glob(O+"bert_*.log")):
    for l in open(f):
        if l.startswith('{"metric"'):
            d=json.loads(l); print(f.split("/")[-1], d["value"], d["p50_ms"], d["p99_ms"])
PY
