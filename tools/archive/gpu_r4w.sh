# round 4: CU-time tile A/B, second pass (o-proj on 256x256; FFN-up on 256x256 / 128x256), then a
# kernel trace of the Llama-3-8B TP=1 bs1 prefill (slower than round 2: find the kernel)
set -o pipefail
rm -f gpurun_out/abt/summary.txt
AB_TABLES=tools/ab_tables_r4w bash tools/gpu_ab_tables.sh 2 || exit $?
mkdir -p gpurun_out/r4w && cp gpurun_out/abt/summary.txt gpurun_out/r4w/tables_ab.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4w/profllama -o l -- \
  python3 bench/llama_tp_bench.py --batches 1 --iters 10 > gpurun_out/r4w/prof_llama.log 2>&1 || exit $?
f=$(ls gpurun_out/r4w/profllama/*/l_kernel_trace.csv gpurun_out/r4w/profllama/l_kernel_trace.csv 2>/dev/null | head -n 1)
python3 bench/trace_table.py "$f" --tail 0.2 --marker rope > gpurun_out/r4w/trace_table_llama_bs1.txt 2>&1
rm -f "$f"
