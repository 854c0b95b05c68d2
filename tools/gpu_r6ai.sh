#!/bin/bash
# Round 6 final tree, every BASELINE config on one MI355X: BERT driver-shaped x10 (the driver's own command) and
# 300 steps x2, dyn-batch <= 16 x2, ResNet-50 closed 128 x2 + Poisson, Llama-3-8B TP=1 serving, and rocprof
# kernel stats of the BERT headline and ResNet-50 serving engines.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6ai
mkdir -p $O
export PYTHONUNBUFFERED=1
for i in 1 2 3 4 5 6 7 8 9 10; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_$i.log 2>&1 || { tail -20 $O/drv_$i.log; exit 1; }
  grep '^{"metric"' $O/drv_$i.log | cut -c1-160
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 300 --warmup 30 > $O/long_$i.log 2>&1 || { tail -20 $O/long_$i.log; exit 1; }
  timeout -k 10 300 python bench.py --steps 300 --warmup 30 --max-batch 16 > $O/b16_$i.log 2>&1 || { tail -20 $O/b16_$i.log; exit 1; }
  timeout -k 10 300 python bench/serve_bench.py --model resnet50 --closed 128 --seconds 5 \
      --json-out $O/rn_c128_$i.json > $O/rn_c128_$i.log 2>&1 || { tail -20 $O/rn_c128_$i.log; exit 1; }
done
timeout -k 10 600 python bench/serve_bench.py --model resnet50 --rates 40000,44000,48000 --seconds 4 \
    --json-out $O/rn_poisson.json > $O/rn_poisson.log 2>&1 || { tail -20 $O/rn_poisson.log; exit 1; }
timeout -k 10 400 python bench/llama_tp_bench.py --serve --loop native --requests 400 --concurrency 16 \
    --json-out $O/llama_tp1.json > $O/llama_tp1.log 2>&1 || { tail -20 $O/llama_tp1.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bert -- python3 bench.py --steps 100 --warmup 10 \
    --json-out $O/bert_prof_bench.json > $O/bert_prof.log 2>&1 || { tail -5 $O/bert_prof.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/resnet -- python3 bench/serve_bench.py --model resnet50 \
    --closed 128 --seconds 3 --json-out $O/resnet_prof_bench.json > $O/resnet_prof.log 2>&1 || { tail -5 $O/resnet_prof.log; exit 1; }
find $O -name "*kernel_trace.csv" -delete
python3 - <<'PY'
import json, glob
O = "gpurun_out/r6ai/"
def line(f):
    return json.loads([l for l in open(f) if l.startswith('{"metric"')][-1])
for pat in ("drv_*.log", "long_*.log", "b16_*.log"):
    for f in sorted(glob.glob(O + pat)):
        d = line(f); print(f.split("/")[-1], d["value"], d["p50_ms"], d["p99_ms"])
for f in sorted(glob.glob(O + "rn_c128_*.json")):
    p = json.load(open(f))["points"][0]; print(f.split("/")[-1], p["req_per_s"], p["p50_ms"], p["p99_ms"])
for p in json.load(open(O + "rn_poisson.json"))["points"]:
    print("rn_poisson", p["offered"], p["req_per_s"], p["p50_ms"], p["p99_ms"])
d = json.load(open(O + "llama_tp1.json")); print("llama_tp1", d["prompts_per_s"], d["p50_ms"], d["p99_ms"], d["mean_batch"])
PY
