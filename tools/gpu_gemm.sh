set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ops.log 2>&1 && \
timeout -k 10 120 python -u bench/bert_breakdown.py --batch 32 > gpurun_out/bd_plain.log 2>&1 && \
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/bd2 -o bd -- python3 bench/bert_breakdown.py --batch 32 --iters 20 > gpurun_out/bd_prof.log 2>&1 && \
timeout -k 10 200 python -u bench.py > gpurun_out/bench_sk.log 2>&1
