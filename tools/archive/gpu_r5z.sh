set -o pipefail
# Round 5: the 256x224 ping-pong tile (cfg 29) -- GEMM tests, then the
# Llama-3-8B TP=1 prefill (start-up tuning sees it for the SwiGLU gate-up) and
# a kernel trace of the bs8 prefill.
bash tools/fresh.sh || exit 9
O=gpurun_out/r5z
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ops_gpu.py -k "linear or tile" > $O/pytest.log 2>&1 || exit $?
timeout -k 10 600 python3 -u bench/llama_tp_bench.py --json-out $O/llama3_8b_tp1_prefill.json > $O/llama_tp1.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/llama_trace -o t -- python3 bench/llama_tp_bench.py --batches 8 --iters 5 > $O/llama_trace.log 2>&1
rc=$?
find $O -type f -size +6M -delete
exit $rc
