set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_models_gpu.py tests/test_models2_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "attention or bert or llama or vit" > gpurun_out/pytest_attn.log 2>&1 && \
timeout -k 10 60 python -u bench/attn_probe.py > gpurun_out/attn_probe.log 2>&1 && \
timeout -k 10 60 python -u bench/attn_probe.py --b 8 --s 512 --h 32 --hkv 8 --d 128 --causal >> gpurun_out/attn_probe.log 2>&1 && \
timeout -k 10 120 python -u bench/bert_breakdown.py --batch 32 > gpurun_out/bd_plain.log 2>&1 && \
timeout -k 10 200 python -u bench.py > gpurun_out/bench_attn.log 2>&1
