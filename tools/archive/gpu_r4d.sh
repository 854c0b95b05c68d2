# round 4: new GPU tests (softmax_topk, stream-K GEMM, TP at real dims, RCCL world 1),
# ablation bounds + idle-dispatch A/B, serving curves of both batch policies, TP8 rehearsal
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r4d
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 ./labbin/pp32_lab --iters 50 > gpurun_out/r4d/pp32_lab.txt 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_ops_gpu.py -k "softmax_topk or streamk" > gpurun_out/r4d/pytest_ops.log 2>&1 || exit $?
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_tp_real_dims_gpu.py > gpurun_out/r4d/pytest_tp.log 2>&1 || exit $?
bash tools/gpu_ab_env.sh 2 "RDB_AB=0" "RDB_ABLATE=ln" "RDB_ABLATE=gelu" "RDB_AB=0 -- --batch-policy idle" || exit $?
for pol in timeout idle; do
  for r in 5000 10000 20000 28000; do
    timeout -k 10 150 python -u bench.py --rate $r --steps 300 --warmup 30 --batch-policy $pol --json-out gpurun_out/r4d/curve_${pol}_$r.json > gpurun_out/r4d/curve_${pol}_$r.log 2>&1 || exit $?
  done
done
timeout -k 10 600 python -u bench/llama_tp8_rehearsal.py --world 8 --json-out gpurun_out/r4d/llama3_8b_tp8_rehearsal.json > gpurun_out/r4d/rehearsal.log 2>&1
