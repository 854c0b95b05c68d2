set -o pipefail
# Round 5: throughput vs p99 serving curve on one MI355X (Poisson open loop at
# fixed offered rates + closed loop), both batch policies.
bash tools/fresh.sh || exit 9
O=gpurun_out/r5s
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for pol in timeout idle; do
  for rate in 5000 10000 20000 28000 32000; do
    steps=$(( rate / 32 / 2 ))   # ~0.5 s of offered load at >= 150 steps
    [ $steps -lt 150 ] && steps=150
    timeout -k 10 200 python3 bench.py --rate $rate --steps $steps --warmup 20 --batch-policy $pol --json-out $O/${pol}_r$rate.json > /dev/null 2>&1 || exit $?
  done
  timeout -k 10 200 python3 bench.py --steps 2000 --warmup 50 --batch-policy $pol --json-out $O/${pol}_closed.json > /dev/null 2>&1 || exit $?
done
