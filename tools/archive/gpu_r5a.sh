set -o pipefail
# Round 5, first GPU call: driver-shaped bench on this tree, then the
# hipBLASLt-vs-ours GEMM side-by-side (timing, vendor kernel names, counters).
bash tools/fresh.sh || exit 9
O=gpurun_out/r5a
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err && \
timeout -k 10 300 python3 bench.py --gpus 1 --steps 2000 --warmup 50 > $O/bench_2000.json 2> $O/bench_2000.err && \
timeout -k 10 300 python3 bench/gemm_vendor_probe.py --which both --sweep > $O/gemm_side_by_side.jsonl 2> $O/gemm_side_by_side.err && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt_vendor -o p -- python3 bench/gemm_vendor_probe.py --which vendor --iters 20 > $O/kt_vendor.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt_ours -o p -- python3 bench/gemm_vendor_probe.py --which ours --iters 20 > $O/kt_ours.log 2>&1
rc=$?
find $O -name "*.csv" -size +4M -delete
exit $rc
