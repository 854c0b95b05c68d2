set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "linear_ln or bert" > gpurun_out/fold_tests.log 2>&1 && \
timeout -k 10 120 python -u bench/bert_breakdown.py --batch 32 > gpurun_out/fold_bd_on.log 2>&1 && \
RDB_BERT_FOLD_LN=0 timeout -k 10 120 python -u bench/bert_breakdown.py --batch 32 > gpurun_out/fold_bd_off.log 2>&1 && \
timeout -k 10 200 python -u bench.py > gpurun_out/fold_bench_on.log 2>&1 && \
RDB_BERT_FOLD_LN=0 timeout -k 10 200 python -u bench.py > gpurun_out/fold_bench_off.log 2>&1 && \
timeout -k 10 200 python -u bench.py > gpurun_out/fold_bench_on2.log 2>&1
