# N-round tile-table A/B over tools/ab_tables/*.json (bench.py --steps 2000); usage: bash tools/gpu_ab_tables.sh ROUNDS [bench flags]
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/abt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
R=$1; shift
for r in $(seq 1 $R); do
  for t in ${AB_TABLES:-tools/archive/ab_tables}/*.json; do
    n=$(basename $t .json)
    timeout -k 10 150 python -u bench.py --steps 2000 --warmup 50 --tile-table $t "$@" > gpurun_out/abt/${n}_r$r.log 2>&1
    rc=$?
    echo "$n r$r rc=$rc $(tail -n 1 gpurun_out/abt/${n}_r$r.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["p99_ms"])' 2>/dev/null)" >> gpurun_out/abt/summary.txt
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
