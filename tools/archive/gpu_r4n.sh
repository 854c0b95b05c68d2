# round 4 BERT evidence: kernel trace of the headline bench (per-forward table, kernel sum),
# per-kernel hardware counters of one bs32 forward, and a driver-shaped short bench run
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r4n
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4n/prof -o b -- \
  python3 bench.py --steps 2000 --warmup 50 > gpurun_out/r4n/bench_prof.log 2>&1 || exit $?
f=$(ls gpurun_out/r4n/prof/*/b_kernel_trace.csv gpurun_out/r4n/prof/b_kernel_trace.csv 2>/dev/null | head -n 1)
python3 bench/trace_table.py "$f" --tail 0.3 > gpurun_out/r4n/trace_table_bench.txt 2>&1
python3 bench/trace_gaps.py "$f" --tail 0.3 > gpurun_out/r4n/trace_gaps_bench.txt 2>&1
s=$(ls gpurun_out/r4n/prof/*/b_kernel_stats.csv gpurun_out/r4n/prof/b_kernel_stats.csv 2>/dev/null | head -n 1)
cp "$s" gpurun_out/r4n/kernel_stats.csv
rm -f "$f"
bash tools/gpu_pmc_r4_bert.sh || exit $?
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4n/bench_driver_shape.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 2000 --warmup 50 > gpurun_out/r4n/bench_long.log 2>&1 || exit $?
# the 8-rank protocol with the uniform pow-2 second sample (round 3 saw alternating per-replica counts)
timeout -k 10 300 python -u bench.py --gpus 8 --rehearse-one-gpu --steps 40 --warmup 5 > gpurun_out/r4n/rehearsal_8.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --gpus 4 --rehearse-one-gpu --steps 40 --warmup 5 > gpurun_out/r4n/rehearsal_4.log 2>&1 || exit $?
# ResNet-50 forward with the fused stem: per-forward kernel table (kernel sum) and single-stream time
T=ray_dynamic_batching_amd/ops/tuned/mi355x_resnet50_B32_cs2_d4.json
timeout -k 10 200 python -u bench/cnn_breakdown.py --model resnet50 --batch 32 --iters 30 --tune-file $T > gpurun_out/r4n/cnn_breakdown.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4n/profcnn -o c -- \
  python3 bench/cnn_breakdown.py --model resnet50 --batch 32 --iters 20 --tune-file $T > gpurun_out/r4n/prof_cnn.log 2>&1 || exit $?
f=$(ls gpurun_out/r4n/profcnn/*/c_kernel_trace.csv gpurun_out/r4n/profcnn/c_kernel_trace.csv 2>/dev/null | head -n 1)
python3 bench/trace_table.py "$f" --tail 0.5 --marker softmax_topk > gpurun_out/r4n/trace_table_resnet_forward.txt 2>&1
rm -f "$f"
