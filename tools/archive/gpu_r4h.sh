# round 4: config 5 with live re-planning (GPU test + duty / priority runs of
# bench/colocation_replan_bench.py)
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r4h
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_colocation_replan_gpu.py \
  > gpurun_out/r4h/pytest_replan.log 2>&1 || exit $?
timeout -k 10 200 python -u bench/colocation_replan_bench.py --slots 2 --policy duty --json-out gpurun_out/r4h/replan_duty.json \
  > gpurun_out/r4h/replan_duty.log 2>&1 || exit $?
timeout -k 10 200 python -u bench/colocation_replan_bench.py --slots 2 --policy priority --json-out gpurun_out/r4h/replan_priority.json \
  > gpurun_out/r4h/replan_priority.log 2>&1
