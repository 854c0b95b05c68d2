set -o pipefail
# Round 5: engine stream stagger (RDB_ENGINE_STAGGER_US) vs lockstep, steady
# state and the driver-shaped window, interleaved.
bash tools/fresh.sh || exit 9
O=gpurun_out/r5ab
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for st in 0 500 900; do
    RDB_ENGINE_STAGGER_US=$st timeout -k 10 200 python3 bench.py --steps 2000 --warmup 50 --json-out $O/s2000_st${st}_r$r.json > /dev/null 2>&1 || exit $?
  done
done
for r in 1 2; do
  for st in 0 500 900; do
    RDB_ENGINE_STAGGER_US=$st timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --json-out $O/s20_st${st}_r$r.json > /dev/null 2>&1 || exit $?
  done
done
