# full-row GEMM+LayerNorm: kernel tests, probe, then a 3-round bench A/B over RDB_BERT_ROWLN
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r3j
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -k "rowln" -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider -m gpu > gpurun_out/r3j/pytest.log 2>&1 || exit $?
timeout -k 10 120 python -u bench/rowln_probe.py --tune-file ray_dynamic_batching_amd/ops/tuned/mi355x_bert_L12_S128_B32_cs2_d4.json > gpurun_out/r3j/probe.json 2>&1 || exit $?
for r in 1 2 3; do
  for m in 0 1 o d; do
    RDB_BERT_ROWLN=$m timeout -k 10 150 python -u bench.py --steps 2000 --warmup 50 > gpurun_out/r3j/rowln_${m}_r$r.log 2>&1
    rc=$?
    echo "$m r$r rc=$rc $(tail -n 1 gpurun_out/r3j/rowln_${m}_r$r.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["p99_ms"])' 2>/dev/null)" >> gpurun_out/r3j/summary.txt
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
