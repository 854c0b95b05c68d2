set -o pipefail
mkdir -p gpurun_out

timeout -k 10 600 python -u -m pytest tests/test_tp8_gpu.py -x -v --timeout 500 --timeout-method thread -p no:cacheprovider -s -k "llama or replica" > gpurun_out/tp8b.log 2>&1
