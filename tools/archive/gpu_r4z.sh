# round 4: last CU-time pass on the headline bench (FFN-up on the BK64 ping-pong 256x128, QKV+attention at bs32
# with two sequences per block), then a kernel trace of the final shipped configuration
set -o pipefail
rm -f gpurun_out/abt/summary.txt
AB_TABLES=tools/ab_tables_r4z bash tools/gpu_ab_tables.sh 2 || exit $?
mkdir -p gpurun_out/r4z && cp gpurun_out/abt/summary.txt gpurun_out/r4z/tables_ab.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4z/prof -o b -- \
  python3 bench.py --steps 2000 --warmup 50 > gpurun_out/r4z/bench_prof.log 2>&1 || exit $?
f=$(ls gpurun_out/r4z/prof/*/b_kernel_trace.csv gpurun_out/r4z/prof/b_kernel_trace.csv 2>/dev/null | head -n 1)
python3 bench/trace_table.py "$f" --tail 0.3 --marker embed16 > gpurun_out/r4z/trace_table_bench.txt 2>&1
python3 bench/trace_gaps.py "$f" --tail 0.3 > gpurun_out/r4z/trace_gaps_bench.txt 2>&1
rm -f "$f"
