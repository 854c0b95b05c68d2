set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u bench.py > gpurun_out/bench_ctx1.log 2>&1 && \
RDB_TUNE_IN_CONTEXT=0 timeout -k 10 200 python -u bench.py > gpurun_out/bench_ctx0.log 2>&1 && \
timeout -k 10 200 python -u bench.py > gpurun_out/bench_ctx1b.log 2>&1 && \
RDB_TUNE_IN_CONTEXT=0 timeout -k 10 200 python -u bench.py > gpurun_out/bench_ctx0b.log 2>&1
