set -o pipefail
# Round 5: ResNet-50 table tuned with the VGPR-staged tiles among the 1x1-conv
# (CONV_LINEAR) candidates vs the shipped table, interleaved.
bash tools/fresh.sh || exit 9
O=gpurun_out/r5p
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$GRAFT_REPO_ROOT/$O/resnet_v4_table.json
rm -f $T
RDB_TUNE_FILE=$T timeout -k 10 600 python3 bench/serve_bench.py --model resnet50 --closed 96 --seconds 8 --json-out $O/tune.json > $O/tune.out 2>&1 || exit $?
for r in 1 2 3; do
  RDB_TUNE_FILE=$T timeout -k 10 300 python3 bench/serve_bench.py --model resnet50 --closed 96 --seconds 8 --json-out $O/new_r$r.json > $O/new_r$r.out 2>&1 || exit $?
  timeout -k 10 300 python3 bench/serve_bench.py --model resnet50 --closed 96 --seconds 8 --json-out $O/old_r$r.json > $O/old_r$r.out 2>&1 || exit $?
done
