set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "linear or skinny or conv" > gpurun_out/pytest_ops.log 2>&1 && \
timeout -k 10 120 python -u bench/gemm_probe.py --m 4096 --n 2304 --k 768 --bias --iters 100 > gpurun_out/probe2.jsonl 2>&1 && \
timeout -k 10 120 python -u bench/gemm_probe.py --m 4096 --n 768 --k 768 --bias --res --iters 100 >> gpurun_out/probe2.jsonl 2>&1 && \
timeout -k 10 120 python -u bench/gemm_probe.py --m 4096 --n 3072 --k 768 --bias --act gelu --iters 100 >> gpurun_out/probe2.jsonl 2>&1 && \
timeout -k 10 120 python -u bench/gemm_probe.py --m 4096 --n 768 --k 3072 --bias --res --iters 100 >> gpurun_out/probe2.jsonl 2>&1 && \
timeout -k 10 120 python -u bench/gemm_probe.py --m 4096 --n 4096 --k 4096 --iters 50 >> gpurun_out/probe2.jsonl 2>&1 && \
timeout -k 10 120 python -u bench/bert_breakdown.py --batch 32 > gpurun_out/bd_plain.log 2>&1
