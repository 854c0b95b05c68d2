#!/bin/bash
# Round 6 closing: ResNet-50 single-stream tables re-tuned after the halo patch swizzle (two tunings,
# RDB_TUNE_STREAMS=1) vs the shipped cs1 table, graph replay interleaved x2; rocprof kernel table of the best.
set -o pipefail
O=gpurun_out/r6ay
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export RDB_TUNE_STREAMS=1
S=ray_dynamic_batching_amd/ops/tuned/mi355x_resnet50_B32_cs1_d2.json
cp $S $O/s.json
for t in a b; do
  rm -f $O/$t.json
  timeout -k 10 400 python -u bench/cnn_breakdown.py --model resnet50 --batch 32 --iters 30 --tune-file $O/$t.json > $O/tune_$t.log 2>&1 || { tail -20 $O/tune_$t.log; exit 1; }
done
for i in 1 2; do
  for t in s a b; do
    timeout -k 10 200 python -u bench/cnn_breakdown.py --model resnet50 --batch 32 --iters 100 --tune-file $O/$t.json > $O/replay_${t}_$i.log 2>&1 || { tail -20 $O/replay_${t}_$i.log; exit 1; }
    echo "$t $i $(grep '^{' $O/replay_${t}_$i.log | tail -n 1)"
  done
done
best=$(python3 - <<'PY'
import json
O="gpurun_out/r6ay/"
def ms(t): return sum(json.loads([l for l in open(f"{O}replay_{t}_{i}.log") if l.startswith("{")][-1])["ms_per_forward"] for i in (1,2))
print(min(("s","a","b"), key=ms))
PY
)
echo "best $best"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c -- \
  python3 bench/cnn_breakdown.py --model resnet50 --batch 32 --iters 20 --tune-file $O/$best.json > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(ls $O/prof/*/c_kernel_trace.csv $O/prof/c_kernel_trace.csv 2>/dev/null | head -n 1)
python3 bench/trace_table.py "$f" --tail 0.5 --marker softmax_topk > $O/trace_table_resnet_forward_cs1.txt 2>&1
rm -f "$f"
head -3 $O/trace_table_resnet_forward_cs1.txt
