# 256x192 ping-pong tiles (cfg 24/25): numerics, standalone FFN-up timing, same-box bench A/B vs the shipped table
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r3s
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "linear" > gpurun_out/r3s/pytest_linear.log 2>&1 || exit $?
for c in 22 23 24 25; do
  timeout -k 10 120 python -u bench/gemm_probe.py --m 4096 --n 3072 --k 768 --cfg $c --act gelu --bias --iters 300 >> gpurun_out/r3s/probe.log 2>&1 || exit $?
done
T=$GRAFT_REPO_ROOT/tools/ab_tables_r3s
bash tools/gpu_ab_env.sh 3 "RDB_AB_SHIPPED=1" "RDB_TUNE_FILE=$T/ffn1_cfg24.json" "RDB_TUNE_FILE=$T/ffn1_cfg25.json"
