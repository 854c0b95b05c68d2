set -o pipefail
# Round 5: ping-pong implicit-GEMM conv tiles (CONV_PP): numerics, a tile table
# tuned with them, same-box A/B against the shipped ResNet-50 table, a kernel
# trace of one bs32 forward.
bash tools/fresh.sh || exit 9
O=gpurun_out/r5f
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$GRAFT_REPO_ROOT/$O/resnet_pp_table.json
rm -f $T
echo "start $(date +%T)" > $O/progress.txt
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ops_gpu.py tests/test_ln_staged_gpu.py -k "conv2d or splitk or streamk or rowln or residual_ln or staged or partial" > $O/pytest_conv.log 2>&1 && echo "pytest ok $(date +%T)" >> $O/progress.txt && \
RDB_TUNE_FILE=$T timeout -k 10 600 python3 -u bench/serve_bench.py --model resnet50 --closed 96 --seconds 8 --json-out $O/resnet_tune.json > $O/resnet_tune.out 2> $O/resnet_tune.err && echo "tune ok $(date +%T)" >> $O/progress.txt && \
RDB_TUNE_FILE=$T timeout -k 10 300 python3 bench/serve_bench.py --model resnet50 --closed 96 --seconds 8 --json-out $O/resnet_new_r1.json > $O/resnet_new_r1.out 2>&1 && \
timeout -k 10 300 python3 bench/serve_bench.py --model resnet50 --closed 96 --seconds 8 --json-out $O/resnet_old_r1.json > $O/resnet_old_r1.out 2>&1 && \
RDB_TUNE_FILE=$T timeout -k 10 300 python3 bench/serve_bench.py --model resnet50 --closed 96 --seconds 8 --json-out $O/resnet_new_r2.json > $O/resnet_new_r2.out 2>&1 && \
timeout -k 10 300 python3 bench/serve_bench.py --model resnet50 --closed 96 --seconds 8 --json-out $O/resnet_old_r2.json > $O/resnet_old_r2.out 2>&1 && echo "ab ok $(date +%T)" >> $O/progress.txt && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_new -o t -- python3 bench/cnn_breakdown.py --model resnet50 --batch 32 --iters 20 --tune-file $T > $O/trace_new.log 2>&1
rc=$?
echo "end rc=$rc $(date +%T)" >> $O/progress.txt
find $O -type f -size +4M -delete
du -sh $O >> $O/progress.txt
exit $rc
