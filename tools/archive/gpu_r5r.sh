set -o pipefail
# Round 5 (final tree): whole GPU test suite + smoke, then the 8-rank rehearsal
# of bench.py (8 ranks on one GPU over gloo: protocol check, not a measurement).
bash tools/fresh.sh || exit 9
O=gpurun_out/r5r
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --maxfail=10 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?
tail -3 $O/pytest_gpu.log > $O/summary.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --gpus 8 --rehearse-one-gpu --steps 30 --warmup 5 > $O/rehearse8.out 2> $O/rehearse8.err
