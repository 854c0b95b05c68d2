# Same-box A/B of environment settings on the headline bench (shipped tile table).
# Usage: bash tools/gpu_ab_env.sh ROUNDS "ARGS_A" "ARGS_B" ...   (each ARGS: env assignments and/or -- bench flags)
# An arm "X=1 Y=2 -- --compute-streams 3" sets env X, Y and passes --compute-streams 3.
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/abe
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
R=$1; shift
for r in $(seq 1 $R); do
  i=0
  for arm in "$@"; do
    i=$((i+1))
    envs="${arm%%--*}"; flags=""
    case "$arm" in *--*) flags="${arm#*--}";; esac
    timeout -k 10 150 env $envs RDB_AB_ARM=$i python -u bench.py --steps 2000 --warmup 50 $flags > gpurun_out/abe/arm${i}_r$r.log 2>&1
    rc=$?
    echo "arm$i [$arm] r$r rc=$rc $(tail -n 1 gpurun_out/abe/arm${i}_r$r.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["p99_ms"])' 2>/dev/null)" >> gpurun_out/abe/summary.txt
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
