# round 4: config 4 refresh with SwiGLU on the ping-pong tiles -- TP1 serving through the shm rings, TP8 rehearsal
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r4s
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u bench/llama_tp_bench.py --serve --json-out gpurun_out/r4s/llama3_8b_tp1_serve_r4.json \
  > gpurun_out/r4s/serve.log 2>&1 || exit $?
timeout -k 10 600 python -u bench/llama_tp8_rehearsal.py --world 8 --json-out gpurun_out/r4s/llama3_8b_tp8_rehearsal_r4.json \
  > gpurun_out/r4s/rehearsal.log 2>&1
