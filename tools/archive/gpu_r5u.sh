set -o pipefail
# Round 5: block-stamp timeline of the UN-profiled ResNet-50 closed loop.
bash tools/fresh.sh || exit 9
O=gpurun_out/r5u
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=$GRAFT_REPO_ROOT/ray_dynamic_batching_amd/_variants/stamps/_rdb_ops.cpython-310-x86_64-linux-gnu.so
RDB_OPS_SO=$V timeout -k 10 300 python3 bench/serve_bench.py --model resnet50 --closed 96 --stamps-out $O/st_resnet.npy --json-out $O/resnet_stamped.json > $O/resnet.out 2>&1 && \
timeout -k 10 300 python3 bench/stamp_timeline.py $O/st_resnet.npy -o $O/tl_resnet.json > /dev/null 2>&1
rc=$?
rm -f $O/st_resnet.npy
exit $rc
