# Reproduce the round-2 ordering (ops kernel tests, then the xGMI graph-replay test, ONE process)
# with plain norm stores, once with SDMA readback and once with blit-kernel copies.
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/xg
T="timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_xgmi_gpu.py -v --timeout 120 --timeout-method thread -p no:cacheprovider -k"
K="linear or norms or embed or qkv_attention or graph_replay"
RDB_XGMI_NORM_STORE=0 RDB_XGMI_DIAG_FILE=gpurun_out/xg/diag2_plain_sdma.jsonl $T "$K" > gpurun_out/xg/order_plain_sdma.log 2>&1; echo "order_plain_sdma rc=$?" >> gpurun_out/xg/status2.txt
RDB_XGMI_NORM_STORE=0 HSA_ENABLE_SDMA=0 RDB_XGMI_DIAG_FILE=gpurun_out/xg/diag2_plain_blit.jsonl $T "$K" > gpurun_out/xg/order_plain_blit.log 2>&1; echo "order_plain_blit rc=$?" >> gpurun_out/xg/status2.txt
