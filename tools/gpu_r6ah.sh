#!/bin/bash
# Round 6 (late): the driver round-end GPU tier on this tree (SDMA input copy, capture split-K workspace, graphs-on TP rehearsal): smoke + pytest -m gpu.
set -o pipefail
O=gpurun_out/r6ah
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 1050 python -u -m pytest tests/ -q -m gpu --maxfail=5 --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/pytest_gpu.log 2>&1
rc=$?
tail -15 $O/pytest_gpu.log
[ $rc = 0 ] || exit $rc
timeout -k 10 200 python -u bench/bert_breakdown.py --batch 32 --iters 100 --tune-file ray_dynamic_batching_amd/ops/tuned/mi355x_bert_L12_S128_B32_cs1_d2.json > $O/bert_cs1.log 2>&1 || { tail -20 $O/bert_cs1.log; exit 1; }
grep '^{' $O/bert_cs1.log | tail -n 1

