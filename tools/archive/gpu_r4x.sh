# round 4: split-K on the dense GEMM (linear): numerics, Llama-3-8B TP=1 prefill with the new candidates,
# and the headline bench on the updated BERT table (o-proj on the 256x128 ping-pong tile)
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r4x
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ops_gpu.py \
  -k "linear or splitk or deep" > gpurun_out/r4x/pytest.log 2>&1 || exit $?
timeout -k 10 600 python -u bench/llama_tp_bench.py --json-out gpurun_out/r4x/llama3_8b_tp1_prefill_r4.json \
  > gpurun_out/r4x/llama_tp1.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4x/bench_driver_shape.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 2000 --warmup 50 > gpurun_out/r4x/bench_long.log 2>&1
