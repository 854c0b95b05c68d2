set -o pipefail
# Round 5: the library built with VGPR-form MFMA accumulators (no AGPR copies in
# the DEEP / big 4-wave tiles) -- correctness of every tile, then ResNet-50 and
# BERT tables tuned on it vs the shipped tables on the default build.
bash tools/fresh.sh || exit 9
O=gpurun_out/r5j
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=$GRAFT_REPO_ROOT/ray_dynamic_batching_amd/_variants/vgprform/_rdb_ops.cpython-310-x86_64-linux-gnu.so
TR=$GRAFT_REPO_ROOT/$O/resnet_vf_table.json
TB=$GRAFT_REPO_ROOT/$O/bert_vf_table.json
rm -f $TR $TB
echo "start $(date +%T)" > $O/progress.txt
RDB_OPS_SO=$V timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ops_gpu.py -k "tile or deep or conv2d or linear" > $O/pytest_vf.log 2>&1 && echo "pytest ok $(date +%T)" >> $O/progress.txt && \
RDB_OPS_SO=$V timeout -k 10 400 python3 bench/conv_probe.py --json-out $O/conv_probe_vf.json > $O/conv_probe_vf.txt 2>&1 && \
RDB_OPS_SO=$V RDB_TUNE_FILE=$TR timeout -k 10 600 python3 bench/serve_bench.py --model resnet50 --closed 96 --seconds 8 --json-out $O/resnet_vf_tune.json > $O/resnet_vf_tune.out 2>&1 && echo "resnet tune ok $(date +%T)" >> $O/progress.txt && \
for r in 1 2; do
  RDB_OPS_SO=$V RDB_TUNE_FILE=$TR timeout -k 10 300 python3 bench/serve_bench.py --model resnet50 --closed 96 --seconds 8 --json-out $O/resnet_vf_r$r.json > $O/resnet_vf_r$r.out 2>&1 || exit $?
  timeout -k 10 300 python3 bench/serve_bench.py --model resnet50 --closed 96 --seconds 8 --json-out $O/resnet_old_r$r.json > $O/resnet_old_r$r.out 2>&1 || exit $?
done && echo "resnet ab ok $(date +%T)" >> $O/progress.txt && \
RDB_OPS_SO=$V RDB_TUNE_FILE=$TB timeout -k 10 400 python3 bench.py --steps 2000 --warmup 50 --json-out $O/bert_vf_tune.json > $O/bert_vf_tune.out 2>&1 && \
for r in 1 2; do
  RDB_OPS_SO=$V RDB_TUNE_FILE=$TB timeout -k 10 300 python3 bench.py --steps 2000 --warmup 50 --json-out $O/bert_vf_r$r.json > $O/bert_vf_r$r.out 2>&1 || exit $?
  timeout -k 10 300 python3 bench.py --steps 2000 --warmup 50 --json-out $O/bert_old_r$r.json > $O/bert_old_r$r.out 2>&1 || exit $?
done
rc=$?
echo "end rc=$rc $(date +%T)" >> $O/progress.txt
exit $rc
