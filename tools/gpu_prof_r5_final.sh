# round 5: rocprofv3 kernel traces of the final tree -- the headline bench (two
# streams, steady-state tail) and one single-stream BERT-base bs32 forward
# (graph replays, shipped table)
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r5p
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5p/prof -o b -- \
  python3 bench.py --steps 2000 --warmup 50 > gpurun_out/r5p/bench_prof.log 2>&1 || exit $?
f=$(ls gpurun_out/r5p/prof/*/b_kernel_trace.csv gpurun_out/r5p/prof/b_kernel_trace.csv 2>/dev/null | head -n 1)
python3 bench/trace_table.py "$f" --tail 0.3 --marker embed16 > gpurun_out/r5p/trace_table_bench.txt 2>&1
python3 bench/trace_gaps.py "$f" --tail 0.3 > gpurun_out/r5p/trace_gaps_bench.txt 2>&1
rm -f "$f"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5p/bd -o bd -- \
  python3 bench/bert_breakdown.py --batch 32 --iters 50 --tune-file ray_dynamic_batching_amd/ops/tuned/mi355x_bert_L12_S128_B32_cs2_d4.json \
  > gpurun_out/r5p/breakdown.log 2>&1 || exit $?
f=$(ls gpurun_out/r5p/bd/*/bd_kernel_trace.csv gpurun_out/r5p/bd/bd_kernel_trace.csv 2>/dev/null | head -n 1)
python3 bench/trace_table.py "$f" --tail 0.5 --marker embed16 > gpurun_out/r5p/trace_table_single.txt 2>&1
rm -f "$f"
