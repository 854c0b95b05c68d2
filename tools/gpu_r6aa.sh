#!/bin/bash
# Round 6: engine input copy A/B -- the zero-copy gather_rows kernel (default) vs strided
# hipMemcpy2DAsync of consecutive ring slots (RDB_ENGINE_DMA_GATHER=1), interleaved x3:
# ResNet-50 closed loop 128 (4.8 MB of uint8 images per batch) and the BERT headline engine.
set -o pipefail
O=gpurun_out/r6aa
mkdir -p $O
export PYTHONUNBUFFERED=1
for i in 1 2 3; do
  for arm in gather dma; do
    if [ $arm = dma ]; then export RDB_ENGINE_DMA_GATHER=1; else unset RDB_ENGINE_DMA_GATHER; fi
    timeout -k 10 300 python bench/serve_bench.py --model resnet50 --closed 128 --seconds 5 \
        --json-out $O/rn_${arm}_$i.json > $O/rn_${arm}_$i.log 2>&1 || { tail -20 $O/rn_${arm}_$i.log; exit 1; }
  done
done
for i in 1 2; do
  for arm in gather dma; do
    if [ $arm = dma ]; then export RDB_ENGINE_DMA_GATHER=1; else unset RDB_ENGINE_DMA_GATHER; fi
    timeout -k 10 300 python bench.py --steps 300 --warmup 30 > $O/bert_${arm}_$i.log 2>&1 || { tail -20 $O/bert_${arm}_$i.log; exit 1; }
  done
done
python - <<'PY'
import json, glob
O="gpurun_out/r6aa/"
for f in sorted(glob.glob(O+"rn_*.json")):
    p=json.load(open(f))["points"][0]; print(f.split("/")[-1], p["req_per_s"], p["p50_ms"], p["p99_ms"], p["mean_batch"])
for f in sorted(glob.glob(O+"bert_*.log")):
    for l in open(f):
        if l.startswith('{"metric"'):
            d=json.loads(l); print(f.split("/")[-1], d["value"], d["p50_ms"], d["p99_ms"])
PY
