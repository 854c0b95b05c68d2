# round 4: epilogue-spill fix -- ops/model numerics, then FFN-up tile A/B on the fixed kernels
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r4e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py tests/test_models_gpu.py > gpurun_out/r4e/pytest.log 2>&1 || exit $?
rm -f gpurun_out/abt/summary.txt
AB_TABLES=tools/ab_tables_r4 bash tools/gpu_ab_tables.sh 3
