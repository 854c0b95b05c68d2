set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 200 python -u bench.py > gpurun_out/bench1.log 2>&1 && \
timeout -k 10 200 python -u bench.py --compute-streams 3 > gpurun_out/bench1_s3.log 2>&1
