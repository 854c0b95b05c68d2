#!/bin/bash
# Round 6 final tree: config 5 (ResNet-50 + BERT-base co-located on one GPU, live re-planning under ramping
# Poisson rates) with both engine policies -- the round-5 protocol on the round-6 engine (SDMA copy, halo convs).
set -o pipefail
O=gpurun_out/r6aj
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u bench/colocation_replan_bench.py --slots 2 --policy duty --json-out $O/replan_duty.json \
  > $O/replan_duty.log 2>&1 || { tail -20 $O/replan_duty.log; exit 1; }
timeout -k 10 300 python -u bench/colocation_replan_bench.py --slots 2 --policy priority --json-out $O/replan_priority.json \
  > $O/replan_priority.log 2>&1 || { tail -20 $O/replan_priority.log; exit 1; }
tail -n 5 $O/replan_duty.log; tail -n 5 $O/replan_priority.log
