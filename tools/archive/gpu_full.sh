# whole GPU suite + smoke + a driver-shaped bench run; stops at a timeout/abort/segfault
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/full
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bad() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/full/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/full/status.txt; bad $rc && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> gpurun_out/full/status.txt; bad $rc && exit $rc
timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/full/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/full/status.txt; exit $rc
