set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/cfg
timeout -k 10 400 python -u -m pytest tests/test_tp8_gpu.py -x -v --timeout 380 --timeout-method thread -p no:cacheprovider -s -k "llama_tp8" > gpurun_out/cfg/tp8c.log 2>&1
