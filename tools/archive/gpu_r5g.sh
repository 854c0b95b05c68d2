set -o pipefail
# Round 5: un-profiled concurrency of the BERT bench from in-kernel block stamps
# (diagnostic RDB_BLOCK_STAMPS build), next to a plain run of the same shape.
bash tools/fresh.sh || exit 9
O=gpurun_out/r5g
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=$GRAFT_REPO_ROOT/ray_dynamic_batching_amd/_variants/stamps/_rdb_ops.cpython-310-x86_64-linux-gnu.so
timeout -k 10 300 python3 bench.py --steps 100 --warmup 50 --json-out $O/plain.json > $O/plain.out 2> $O/plain.err && \
RDB_OPS_SO=$V timeout -k 10 300 python3 bench.py --steps 100 --warmup 50 --stamps-out $O/stamps.npy --json-out $O/stamps.json > $O/stamps.out 2> $O/stamps.err && \
timeout -k 10 300 python3 bench/stamp_timeline.py $O/stamps.npy -o $O/stamp_timeline.json > $O/timeline.out 2>&1 && \
python3 -c "import numpy as np; a=np.load('$O/stamps.npy'); np.savez_compressed('$O/stamps_small.npz', rec=a[:200000])"
rc=$?
rm -f $O/stamps.npy
[ $rc -eq 0 ] || exit $rc
# Llama-3-8B TP=1 prefill with the ping-pong split-K candidates (down projection: 128 tiles of 256x128)
timeout -k 10 600 python3 -u bench/llama_tp_bench.py --json-out $O/llama3_8b_tp1_prefill.json > $O/llama_tp1.log 2>&1
rc=$?
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/llama_trace -o t -- python3 bench/llama_tp_bench.py --batches 8 --iters 5 > $O/llama_trace.log 2>&1
rc=$?
find $O -type f -size +6M -delete
exit $rc
