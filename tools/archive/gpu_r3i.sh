# occupancy GEMM lab (solo + 2-stream, stamped) then a driver-shaped bench
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r3i
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 ./labbin/lab_occ --iters 50 --concurrent > gpurun_out/r3i/lab_occ.txt 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3i/bench.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --steps 2000 --warmup 50 > gpurun_out/r3i/bench_long.log 2>&1
