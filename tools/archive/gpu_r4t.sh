# round 4: config 4 at TP = 1 on the round-4 GEMM candidates (DEEP tiles for the small-M prefill GEMMs)
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r4t
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u bench/llama_tp_bench.py --json-out gpurun_out/r4t/llama3_8b_tp1_prefill_r4.json \
  > gpurun_out/r4t/llama_tp1.log 2>&1
