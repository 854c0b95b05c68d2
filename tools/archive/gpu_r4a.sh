# round 4 first look: baseline bench on this box + a kernel trace of the
# headline bench (2-stream overlap per kernel) + the engine tests
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r4a
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 python -u bench.py --steps 400 --warmup 30 > gpurun_out/r4a/bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4a/prof -o b -- \
  python3 bench.py --steps 1500 --warmup 50 > gpurun_out/r4a/bench_prof.log 2>&1 || exit $?
f=$(ls gpurun_out/r4a/prof/*/b_kernel_trace.csv gpurun_out/r4a/prof/b_kernel_trace.csv 2>/dev/null | head -n 1)
python3 bench/trace_gaps.py "$f" --tail 0.3 --timeline gpurun_out/r4a/timeline.txt > gpurun_out/r4a/gaps.txt 2>&1
python3 bench/trace_table.py "$f" --tail 0.3 > gpurun_out/r4a/trace_table.txt 2>&1
rm -f "$f"
timeout -k 10 300 python -u -m pytest tests/test_models2_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4a/pytest_models2.log 2>&1
exit $?
