# BK32 swizzle fix: GEMM numerics over every tile config, then the round-3 PMC passes
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r3r
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "linear or qkv or conv" > gpurun_out/r3r/pytest_ops.log 2>&1 || exit $?
bash tools/gpu_pmc_r3.sh
