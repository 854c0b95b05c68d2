#!/bin/bash
# Round 6 final tree: hardware counters of one bs32 forward (graph replay, single-stream tables) for BERT-base and
# ResNet-50: one rocprofv3 --pmc pass per counter group, then the per-kernel summary (bench/pmc_summary.py).
set -o pipefail
O=gpurun_out/r6ao
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
D=ray_dynamic_batching_amd/ops/tuned
SQ="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE"
for m in bert resnet; do
  if [ $m = bert ]; then
    B="python3 bench/bert_breakdown.py --batch 32 --iters 5 --tune-file $D/mi355x_bert_L12_S128_B32_cs1_d2.json"; MK=embed
  else
    B="python3 bench/cnn_breakdown.py --model resnet50 --batch 32 --iters 5 --tune-file $D/mi355x_resnet50_B32_cs1_d2.json"; MK=softmax_topk
  fi
  timeout -s KILL 240 rocprofv3 --pmc $SQ --output-format csv -d $O/${m}_sq -o p -- $B > $O/${m}_sq.log 2>&1 || { tail -5 $O/${m}_sq.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $O/${m}_fetch -o p -- $B > $O/${m}_fetch.log 2>&1 || { tail -5 $O/${m}_fetch.log; exit 1; }
  python3 bench/pmc_summary.py $O/${m}_sq $O/${m}_fetch -o $O/pmc_${m}_forward_r6.json --marker $MK --forwards 10 --top 30 \
    --note "$m bs32 forward, round-6 final tree, single-stream tile table, graph replay, one counter pass per group (tools/gpu_r6ao.sh)" > $O/${m}_summary.log 2>&1 || { tail -5 $O/${m}_summary.log; exit 1; }
done
find $O -name "*.csv" -size +2M -delete
