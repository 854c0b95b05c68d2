# round 4: SwiGLU on the staged 16-bit epilogue (core + ping-pong tiles): numerics, then config 4 (Llama TP1 prefill)
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r4p
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "swiglu or linear or gemm" > gpurun_out/r4p/pytest_swiglu.log 2>&1 || exit $?
timeout -k 10 600 python -u bench/llama_tp_bench.py --json-out gpurun_out/r4p/llama3_8b_tp1_prefill_r4_swg.json \
  > gpurun_out/r4p/llama_tp1.log 2>&1
