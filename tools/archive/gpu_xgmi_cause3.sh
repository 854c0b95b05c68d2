# the round-2 ordering again, every store flavour, with the priority-separated rank streams
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/xg
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_xgmi_gpu.py -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "linear or norms or embed or qkv_attention or xgmi" > gpurun_out/xg/order_fixed.log 2>&1; echo "order_fixed rc=$?" >> gpurun_out/xg/status3.txt
