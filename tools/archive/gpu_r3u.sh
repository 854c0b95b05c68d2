# residual prefetch in the staged epilogue: GEMM numerics (every tile, residual epilogues) + the residual probe
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r3u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_models_gpu.py -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r3u/pytest.log 2>&1 || exit $?
P="timeout -k 10 120 python -u bench/gemm_probe.py --iters 400 --bias"
$P --m 4096 --n 768 --k 768 --cfg 10 --res > gpurun_out/r3u/o_res.log 2>&1 && \
$P --m 4096 --n 768 --k 3072 --cfg 19 --res > gpurun_out/r3u/d_res.log 2>&1
rc=$?
for f in gpurun_out/r3u/*_res.log; do echo "$f $(grep -o '"ours[^}]*}' $f)"; done
exit $rc
