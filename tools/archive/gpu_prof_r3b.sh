# rocprofv3 kernel trace + stats of the headline bench (shipped tile table), per-forward table
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/prof_r3b
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r3b -o b -- \
  python3 bench.py --steps 3000 --warmup 50 > gpurun_out/prof_r3b/bench.log 2>&1 || exit $?
f=$(ls gpurun_out/prof_r3b/*/b_kernel_trace.csv gpurun_out/prof_r3b/b_kernel_trace.csv 2>/dev/null | head -n 1)
python3 bench/trace_table.py "$f" --tail 0.3 > gpurun_out/prof_r3b/trace_table.txt 2>&1
s=$(ls gpurun_out/prof_r3b/*/b_kernel_stats.csv gpurun_out/prof_r3b/b_kernel_stats.csv 2>/dev/null | head -n 1)
cp "$s" gpurun_out/prof_r3b/kernel_stats.csv
rm -f "$f"
exit 0
