#!/bin/bash
# Round 6: ResNet-50 bs32 single-stream forward on the shipped cs3 table (halo 3x3 convolutions):
# cnn_breakdown timing and a rocprof kernel table per forward (kernel sum).
set -o pipefail
O=gpurun_out/r6z
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=ray_dynamic_batching_amd/ops/tuned/mi355x_resnet50_B32_cs3_d6.json
timeout -k 10 200 python -u bench/cnn_breakdown.py --model resnet50 --batch 32 --iters 30 --tune-file $T > $O/cnn_breakdown.log 2>&1 || { tail -20 $O/cnn_breakdown.log; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c -- \
  python3 bench/cnn_breakdown.py --model resnet50 --batch 32 --iters 20 --tune-file $T > $O/prof_cnn.log 2>&1 || { tail -20 $O/prof_cnn.log; exit 1; }
f=$(ls $O/prof/*/c_kernel_trace.csv $O/prof/c_kernel_trace.csv 2>/dev/null | head -n 1)
python3 bench/trace_table.py "$f" --tail 0.5 --marker softmax_topk > $O/trace_table_resnet_forward.txt 2>&1
rm -f "$f"
cat $O/trace_table_resnet_forward.txt | head -30
tail -5 $O/cnn_breakdown.log
