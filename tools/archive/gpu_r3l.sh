# bs32 A/B: FFN-down tile alternatives (tools/ab_tables) + the full-row GEMM+LayerNorm arms, 2 alternating rounds
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r3l
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {  # name, env assignment, table
  env $2 timeout -k 10 150 python -u bench.py --steps 2000 --warmup 50 --tile-table $3 > gpurun_out/r3l/$1.log 2>&1
  rc=$?
  echo "$1 rc=$rc $(tail -n 1 gpurun_out/r3l/$1.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["p99_ms"])' 2>/dev/null)" >> gpurun_out/r3l/summary.txt
  return $rc
}
for r in 1 2; do
  for t in tools/ab_tables/*.json; do
    run $(basename $t .json)_r$r RDB_BERT_ROWLN=0 $t || exit $?
  done
  run rowln_o_r$r RDB_BERT_ROWLN=o tools/ab_tables/A_shipped.json || exit $?
  run rowln_1_r$r RDB_BERT_ROWLN=1 tools/ab_tables/A_shipped.json || exit $?
done
exit 0
