set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_tp8_gpu.py -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/tp8.log 2>&1
