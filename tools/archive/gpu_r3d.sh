# new GPU tests (device-ring DAG, fp32 parity bound, engine estimates) + smoke, then the tile A/B
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r3d
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_core_dag_gpu.py tests/test_models_fp32_gpu.py "tests/test_models_gpu.py::test_engine_concurrent_streams_match_single_stream" \
  > gpurun_out/r3d/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r3d/status.txt
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3d/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> gpurun_out/r3d/status.txt
case $rc in 124|134|137|139) exit $rc;; esac
bash tools/gpu_ab_tiles.sh
