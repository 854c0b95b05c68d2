set -o pipefail
# Round 5: engine device warm-up (EngineRunner.build, RDB_ENGINE_WARM_S) on the
# driver-shaped window, interleaved with it switched off.
bash tools/fresh.sh || exit 9
O=gpurun_out/r5m
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 1 2 3 4; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --json-out $O/warm_r$r.json > $O/warm_r$r.out 2>&1 || exit $?
  RDB_ENGINE_WARM_S=0 timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --json-out $O/cold_r$r.json > $O/cold_r$r.out 2>&1 || exit $?
done
timeout -k 10 300 python3 bench.py --steps 2000 --warmup 50 --json-out $O/warm_s2000.json > $O/warm_s2000.out 2>&1
