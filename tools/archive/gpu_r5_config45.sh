# round 5 close-out: engine stagger test, config 4 (Llama-3-8B TP1 serving through
# the shm rings) and config 5 (ResNet-50 + BERT co-location with re-planning) on
# the final kernels
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r5y
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  "tests/test_models_gpu.py::test_engine_concurrent_streams_match_single_stream" > gpurun_out/r5y/pytest_stagger.log 2>&1 || exit $?
timeout -k 10 500 python -u bench/llama_tp_bench.py --serve --json-out gpurun_out/r5y/llama3_8b_tp1_serve_r5.json \
  > gpurun_out/r5y/serve.log 2>&1 || exit $?
timeout -k 10 200 python -u bench/colocation_replan_bench.py --slots 2 --policy duty --json-out gpurun_out/r5y/replan_duty.json \
  > gpurun_out/r5y/replan_duty.log 2>&1 || exit $?
timeout -k 10 200 python -u bench/colocation_replan_bench.py --slots 2 --policy priority --json-out gpurun_out/r5y/replan_priority.json \
  > gpurun_out/r5y/replan_priority.log 2>&1
