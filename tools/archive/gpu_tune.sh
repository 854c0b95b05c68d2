set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u bench.py --tune-streams 1 > gpurun_out/bench_t1.log 2>&1 && \
timeout -k 10 200 python -u bench.py --tune-streams 2 > gpurun_out/bench_t2.log 2>&1 && \
timeout -k 10 200 python -u bench.py --tune-streams 3 --compute-streams 3 > gpurun_out/bench_t3.log 2>&1
