# round 4 final tree: the round-end checks (whole GPU suite, smoke) plus the 1-GPU headline bench
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r4q
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
  > gpurun_out/r4q/pytest_gpu_full.log 2>&1 || exit $?
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4q/smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/r4q/bench.log 2>&1
