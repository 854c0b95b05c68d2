# round 4: kernel trace of the Llama-3-8B TP=1 bs8 prefill with SwiGLU on the ping-pong tiles
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r4r
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4r/prof -o l -- \
  python3 bench/llama_tp_bench.py --batches 8 --iters 20 > gpurun_out/r4r/prof_llama.log 2>&1 || exit $?
f=$(ls gpurun_out/r4r/prof/*/l_kernel_trace.csv gpurun_out/r4r/prof/l_kernel_trace.csv 2>/dev/null | head -n 1)
python3 bench/trace_table.py "$f" --tail 0.3 --marker rope > gpurun_out/r4r/trace_table_llama_bs8.txt 2>&1
rm -f "$f"
