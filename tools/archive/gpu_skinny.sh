# Skinny-M GEMM A/B: kernel tests, isolated per-call timing (new vs the _variants/sk_old build),
# then same-box headline A/B (fixed tile table).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OLD=$GRAFT_REPO_ROOT/ray_dynamic_batching_amd/_variants/sk_old/_rdb_ops.cpython-310-x86_64-linux-gnu.so
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -k "skinny or linear" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/sk_tests.log 2>&1 && \
timeout -k 10 120 python -u bench/skinny_probe.py --json gpurun_out/sk_new.json > gpurun_out/sk_new.log 2>&1 && \
timeout -k 10 120 env RDB_OPS_SO=$OLD python -u bench/skinny_probe.py --json gpurun_out/sk_old.json > gpurun_out/sk_old.log 2>&1 && \
bash tools/gpu_ab.sh "RDB_OPS_SO=$OLD" "RDB_AB_NOP=1" 600 > gpurun_out/sk_ab.txt 2>&1
