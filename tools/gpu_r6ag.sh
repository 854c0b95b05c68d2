#!/bin/bash
# Round 6: one split-K workspace (one memset node) per graph capture instead of one per launch -- GPU tests,
# then BERT / ResNet single-stream replays with the cs1 tables and a BERT rocprof kernel table.
set -o pipefail
O=gpurun_out/r6ag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_ops_gpu.py -k "splitk" \
    > $O/pytest_splitk.log 2>&1 || { tail -30 $O/pytest_splitk.log; exit 1; }
tail -2 $O/pytest_splitk.log
T=$1
for i in 1 2; do
  timeout -k 10 200 python -u bench/bert_breakdown.py --batch 32 --iters 100 --tune-file $T > $O/bert_cs1_$i.log 2>&1 || { tail -20 $O/bert_cs1_$i.log; exit 1; }
  echo "bert cs1 $i $(grep '^{' $O/bert_cs1_$i.log | tail -n 1)"
  timeout -k 10 200 python -u bench/cnn_breakdown.py --model resnet50 --batch 32 --iters 100 \
      --tune-file ray_dynamic_batching_amd/ops/tuned/mi355x_resnet50_B32_cs1_d2.json > $O/rn_cs1_$i.log 2>&1 || { tail -20 $O/rn_cs1_$i.log; exit 1; }
  echo "resnet cs1 $i $(grep '^{' $O/rn_cs1_$i.log | tail -n 1)"
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c -- \
  python3 bench/bert_breakdown.py --batch 32 --iters 20 --tune-file $T > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(ls $O/prof/*/c_kernel_trace.csv $O/prof/c_kernel_trace.csv 2>/dev/null | head -n 1)
python3 bench/trace_table.py "$f" --tail 0.5 --marker embed > $O/trace_table_bert_forward_cs1.txt 2>&1
rm -f "$f"
head -20 $O/trace_table_bert_forward_cs1.txt
