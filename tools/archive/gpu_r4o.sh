# round 4: the round-end checks the driver runs -- the whole GPU test suite and smoke() -- on the final tree
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r4o
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
  > gpurun_out/r4o/pytest_gpu_full.log 2>&1 || exit $?
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4o/smoke.log 2>&1
