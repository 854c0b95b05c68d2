set -o pipefail
# Round 5: the whole GPU test suite + smoke on the current tree.
bash tools/fresh.sh || exit 9
O=gpurun_out/r5i
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --maxfail=10 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?
tail -5 $O/pytest_gpu.log > $O/summary.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
