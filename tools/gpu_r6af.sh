#!/bin/bash
# Round 6: BERT-base bs32 single-stream forward with tables tuned for ONE compute stream (two independent
# tunings, RDB_TUNE_STREAMS=1) vs the shipped cs3 table; the faster cs1 table gets a rocprof kernel table.
set -o pipefail
O=gpurun_out/r6af
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export RDB_TUNE_STREAMS=1
for t in a b; do
  rm -f $O/bert_cs1_$t.json
  timeout -k 10 400 python -u bench/bert_breakdown.py --batch 32 --iters 30 --tune-file $O/bert_cs1_$t.json > $O/tune_$t.log 2>&1 || { tail -20 $O/tune_$t.log; exit 1; }
done
S=ray_dynamic_batching_amd/ops/tuned/mi355x_bert_L12_S128_B32_cs3_d6.json
cp $S $O/bert_cs3.json
for i in 1 2; do
  for t in a b cs3; do
    f=$O/bert_cs1_$t.json; [ $t = cs3 ] && f=$O/bert_cs3.json
    timeout -k 10 200 python -u bench/bert_breakdown.py --batch 32 --iters 100 --tune-file $f > $O/replay_${t}_$i.log 2>&1 || { tail -20 $O/replay_${t}_$i.log; exit 1; }
    echo "$t $i $(grep '^{' $O/replay_${t}_$i.log | tail -n 1)"
  done
done
best=$(python3 - <<'PY'
import json
O="gpurun_out/r6af/"
def ms(t): return sum(json.loads([l for l in open(f"{O}replay_{t}_{i}.log") if l.startswith("{")][-1])["ms_per_forward"] for i in (1,2))
print(min(("a","b"), key=ms))
PY
)
echo "best $best"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c -- \
  python3 bench/bert_breakdown.py --batch 32 --iters 20 --tune-file $O/bert_cs1_$best.json > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(ls $O/prof/*/c_kernel_trace.csv $O/prof/c_kernel_trace.csv 2>/dev/null | head -n 1)
python3 bench/trace_table.py "$f" --tail 0.5 --marker embed > $O/trace_table_bert_forward_cs1.txt 2>&1
rm -f "$f"
head -30 $O/trace_table_bert_forward_cs1.txt
