# round 4: tiles with LESS CU-time per GEMM (fewer, bigger blocks: the other stream keeps the rest of the
# GPU): o-proj on the 256x128 / 128x256 ping-pong tiles, FFN-down on 256x256 / 256x192 -- same-box A/B
set -o pipefail
rm -f gpurun_out/abt/summary.txt
AB_TABLES=tools/ab_tables_r4u bash tools/gpu_ab_tables.sh 2 || exit $?
mkdir -p gpurun_out/r4u && cp gpurun_out/abt/summary.txt gpurun_out/r4u/tables_ab.txt
# Llama-3-8B TP=1 prefill with and without the DEEP tile candidates (r4t measured it slower than round 2)
timeout -k 10 600 env RDB_GEMM_DEEP=0 python -u bench/llama_tp_bench.py --json-out gpurun_out/r4u/llama_tp1_nodeep.json \
  > gpurun_out/r4u/llama_nodeep.log 2>&1 || exit $?
timeout -k 10 600 env RDB_GEMM_DEEP=0 RDB_CONV_SPLITK=0 RDB_TUNE_STREAMS=1 python -u bench/llama_tp_bench.py --batches 1,8 \
  --json-out gpurun_out/r4u/llama_tp1_nodeep_ts1.json > gpurun_out/r4u/llama_nodeep_ts1.log 2>&1
