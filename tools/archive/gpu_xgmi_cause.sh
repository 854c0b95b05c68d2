# why did plain stores of the graph-replayed fused norm read back stale?
# 1 baseline plain stores, SDMA readback; 2 plain stores with blit-kernel copies (HSA_ENABLE_SDMA=0);
# 3 write-through default; then the plain-store GEMM readback regression test.
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/xg
T="timeout -k 10 200 python -u -m pytest tests/test_xgmi_gpu.py -v --timeout 120 --timeout-method thread -p no:cacheprovider -k graph_replay"
RDB_XGMI_NORM_STORE=0 RDB_XGMI_DIAG_FILE=gpurun_out/xg/diag_plain_sdma.jsonl $T > gpurun_out/xg/plain_sdma.log 2>&1; echo "plain_sdma rc=$?" >> gpurun_out/xg/status.txt
RDB_XGMI_NORM_STORE=0 HSA_ENABLE_SDMA=0 RDB_XGMI_DIAG_FILE=gpurun_out/xg/diag_plain_blit.jsonl $T > gpurun_out/xg/plain_blit.log 2>&1; echo "plain_blit rc=$?" >> gpurun_out/xg/status.txt
RDB_XGMI_NORM_STORE=1 HSA_ENABLE_SDMA=0 $T > gpurun_out/xg/nt_blit.log 2>&1; echo "nt_blit rc=$?" >> gpurun_out/xg/status.txt
$T > gpurun_out/xg/sc1_sdma.log 2>&1; echo "sc1_sdma rc=$?" >> gpurun_out/xg/status.txt
timeout -k 10 200 python -u -m pytest tests/test_ops_gpu.py -v --timeout 120 --timeout-method thread -p no:cacheprovider -k plain_store_kernel > gpurun_out/xg/gemm_readback.log 2>&1; echo "gemm_readback rc=$?" >> gpurun_out/xg/status.txt
