# bs32 A/B: shipped vs FFN-down / o-proj on tile 23 (two blocks per CU), 3 alternating rounds
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r3p
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {  # name, table, extra args
  timeout -k 10 150 python -u bench.py --steps 2000 --warmup 50 --tile-table $2 $3 > gpurun_out/r3p/$1.log 2>&1
  rc=$?
  echo "$1 rc=$rc $(tail -n 1 gpurun_out/r3p/$1.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["p99_ms"])' 2>/dev/null)" >> gpurun_out/r3p/summary.txt
  return $rc
}
for r in 1 2 3; do
  for t in A_shipped B_ffn2_23 C_oproj_23; do run ${t}_r$r tools/ab_tables_r3p/$t.json "" || exit $?; done
done
exit 0
