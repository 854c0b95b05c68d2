set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_xgmi_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k llama > gpurun_out/pytest_xgmi.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k bert > gpurun_out/pytest_bert.log 2>&1 && \
timeout -k 10 200 python -u bench.py > gpurun_out/bench_cls.log 2>&1
