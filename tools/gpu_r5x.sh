set -o pipefail
# Round 5 (final tree): whole GPU suite + smoke, then the driver-shaped bench
# three times and one steady-state run.
bash tools/fresh.sh || exit 9
O=gpurun_out/r5x
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --maxfail=10 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?
tail -3 $O/pytest_gpu.log > $O/summary.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --json-out $O/driver_r$r.json > $O/driver_r$r.out 2>&1 || exit $?
done
timeout -k 10 200 python3 bench.py --steps 2000 --warmup 50 --json-out $O/steady.json > $O/steady.out 2>&1
