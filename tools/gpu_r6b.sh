#!/bin/bash
# Round 6, second GPU pass: the SURVEY 7.3 slice (@serve.batch ResNet-50 via serve.run),
# Llama-3-8B TP=1 serving on the native engine loop vs the Python loop, ten
# driver-shaped headline runs.
set -o pipefail
O=gpurun_out/r6b
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python bench/serve_batch_slice.py --seconds 8 --concurrency 64 \
    --json-out $O/slice.json > $O/slice.log 2>&1 &&
timeout -k 10 400 python bench/serve_bench.py --model resnet50 --closed 96 --seconds 5 \
    --json-out $O/resnet_direct.json > $O/resnet_direct.log 2>&1 &&
timeout -k 10 400 python bench/llama_tp_bench.py --serve --loop native --requests 400 --concurrency 16 \
    --json-out $O/llama_native.json > $O/llama_native.log 2>&1 &&
timeout -k 10 400 python bench/llama_tp_bench.py --serve --loop python --requests 400 --concurrency 16 \
    --json-out $O/llama_python.json > $O/llama_python.log 2>&1 &&
for i in 1 2 3 4 5 6 7 8 9 10; do
  timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out $O/bench_$i.json > $O/bench_$i.log 2>&1 || exit 1
done
echo "exit $?"
