# round 4: config 5 with live re-planning at >= 70 % of the GPU's measured capacity (phases as
# fractions of it; the planner sees each of --slots executors as 1/slots of the device):
# two executors with the duty cycle and with the priority policy, and one executor (duty)
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r4p
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_colocation_replan_gpu.py \
  > gpurun_out/r4p/pytest_replan.log 2>&1 || exit $?
for arm in "--slots 2 --policy duty" "--slots 2 --policy priority" "--slots 1 --policy duty"; do
  tag=$(echo $arm | tr -d ' -' )
  timeout -k 10 240 python -u bench/colocation_replan_bench.py $arm --json-out gpurun_out/r4p/replan_$tag.json \
    > gpurun_out/r4p/replan_$tag.log 2>&1 || exit $?
done
