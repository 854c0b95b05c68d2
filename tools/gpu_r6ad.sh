#!/bin/bash
# Round 6: ResNet-50 bs32 single-stream forward with a table tuned for ONE stream (halo 3x3 convs among the
# candidates): tune once (RDB_TUNE_STREAMS=1), then graph-replay timing and a rocprof kernel table per forward.
set -o pipefail
O=gpurun_out/r6ad
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$O/resnet50_B32_cs1_tuned.json
rm -f $T
export RDB_TUNE_STREAMS=1
timeout -k 10 400 python -u bench/cnn_breakdown.py --model resnet50 --batch 32 --iters 30 --tune-file $T > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
timeout -k 10 200 python -u bench/cnn_breakdown.py --model resnet50 --batch 32 --iters 50 --tune-file $T > $O/replay.log 2>&1 || { tail -20 $O/replay.log; exit 1; }
S=ray_dynamic_batching_amd/ops/tuned/mi355x_resnet50_B32_cs3_d6.json
timeout -k 10 200 python -u bench/cnn_breakdown.py --model resnet50 --batch 32 --iters 50 --tune-file $S > $O/replay_cs3.log 2>&1 || { tail -20 $O/replay_cs3.log; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c -- \
  python3 bench/cnn_breakdown.py --model resnet50 --batch 32 --iters 20 --tune-file $T > $O/prof_cnn.log 2>&1 || { tail -20 $O/prof_cnn.log; exit 1; }
f=$(ls $O/prof/*/c_kernel_trace.csv $O/prof/c_kernel_trace.csv 2>/dev/null | head -n 1)
python3 bench/trace_table.py "$f" --tail 0.5 --marker softmax_topk > $O/trace_table_resnet_forward_cs1.txt 2>&1
rm -f "$f"
head -40 $O/trace_table_resnet_forward_cs1.txt
tail -2 $O/tune.log $O/replay.log $O/replay_cs3.log
