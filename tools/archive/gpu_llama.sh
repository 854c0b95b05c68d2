set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench/llama_tp_bench.py --json-out gpurun_out/llama_prefill.json > gpurun_out/llama_prefill.log 2>&1 && \
timeout -k 10 400 python -u bench/llama_tp_bench.py --serve --json-out gpurun_out/llama_serve.json > gpurun_out/llama_serve.log 2>&1
