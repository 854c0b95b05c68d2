set -o pipefail
# Round 5: BERT tile table re-tuned with the ping-pong split-K candidates vs the
# shipped table, interleaved same-box runs at --steps 2000.
bash tools/fresh.sh || exit 9
O=gpurun_out/r5h
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$GRAFT_REPO_ROOT/$O/bert_sk_table.json
rm -f $T
timeout -k 10 200 python3 -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_ops_gpu.py -k "private_workspace or linear_splitk" > $O/pytest.log 2>&1 || exit $?
RDB_TUNE_FILE=$T timeout -k 10 300 python3 bench.py --steps 2000 --warmup 50 --json-out $O/tune.json > $O/tune.out 2> $O/tune.err || exit $?
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --steps 2000 --warmup 50 --json-out $O/old_r$r.json > $O/old_r$r.out 2>&1 || exit $?
  RDB_TUNE_FILE=$T timeout -k 10 200 python3 bench.py --steps 2000 --warmup 50 --json-out $O/new_r$r.json > $O/new_r$r.out 2>&1 || exit $?
done
