# round 4: LayerNorm rows per block (8 / 4 / 2: more, smaller blocks) on the headline bench, same box
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py -k "layer_norm or rms or norm" \
  > /dev/null 2>&1 || exit $?
rm -f gpurun_out/abe/summary.txt
bash tools/gpu_ab_env.sh 3 "RDB_AB=0" "RDB_LN_THREADS=128" "RDB_LN_THREADS=64" || exit $?
mkdir -p gpurun_out/r4ee && cp gpurun_out/abe/summary.txt gpurun_out/r4ee/ln_threads_ab.txt
