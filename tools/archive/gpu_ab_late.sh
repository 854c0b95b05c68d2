set -o pipefail
# Round 5: LDS-DMA pieces issued in the matrix interval on the BK-64 ping-pong
# tiles (default build) vs the previous build (RDB_OPS_SO=pre_late), interleaved;
# GEMM / conv tests first; Llama-3-8B prefill once per arm.
bash tools/fresh.sh || exit 9
O=gpurun_out/late_ab
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P=$GRAFT_REPO_ROOT/ray_dynamic_batching_amd/_variants/pre_late/_rdb_ops.cpython-310-x86_64-linux-gnu.so
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ops_gpu.py -k "linear or tile or conv2d" > $O/pytest.log 2>&1 || exit $?
for r in 1 2 3 4 5; do
  timeout -k 10 200 python3 bench.py --steps 2000 --warmup 50 --json-out $O/new_r$r.json > /dev/null 2>&1 || exit $?
  RDB_OPS_SO=$P timeout -k 10 200 python3 bench.py --steps 2000 --warmup 50 --json-out $O/old_r$r.json > /dev/null 2>&1 || exit $?
done
for r in 1 2; do
  timeout -k 10 300 python3 bench/serve_bench.py --model resnet50 --closed 96 --seconds 8 --json-out $O/rn_new_r$r.json > /dev/null 2>&1 || exit $?
  RDB_OPS_SO=$P timeout -k 10 300 python3 bench/serve_bench.py --model resnet50 --closed 96 --seconds 8 --json-out $O/rn_old_r$r.json > /dev/null 2>&1 || exit $?
done
timeout -k 10 600 python3 -u bench/llama_tp_bench.py --batches 8 --json-out $O/llama_new.json > $O/llama_new.log 2>&1 || exit $?
RDB_OPS_SO=$P timeout -k 10 600 python3 -u bench/llama_tp_bench.py --batches 8 --json-out $O/llama_old.json > $O/llama_old.log 2>&1
