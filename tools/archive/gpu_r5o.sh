set -o pipefail
# Round 5: the 4-wave VGPR-staged tiles (cfg 26..28) -- numerics, the standalone
# side-by-side with hipBLASLt (every tile), and a same-box BERT A/B of the
# shipped table vs the same table with o-proj / FFN-down on cfg 26.
bash tools/fresh.sh || exit 9
O=gpurun_out/r5o
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
echo "start $(date +%T)" > $O/progress.txt
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ops_gpu.py -k "linear or tile" > $O/pytest.log 2>&1 && echo "pytest ok $(date +%T)" >> $O/progress.txt || exit $?
timeout -k 10 400 python3 bench/gemm_vendor_probe.py --sweep > $O/probe.txt 2> $O/probe.err || exit $?
echo "probe ok $(date +%T)" >> $O/progress.txt
S=ray_dynamic_batching_amd/ops/tuned/mi355x_bert_L12_S128_B32_cs2_d4.json
python3 - "$S" $O <<'PY'
import json, sys
src, out = sys.argv[1], sys.argv[2]
t = json.load(open(src))
def variant(changes, path):
    v = []
    for k, c in t:
        if k[0] == "gemm" and k[2] == 4096 and (k[3], k[4]) in changes and k[6] == "none":
            c = changes[(k[3], k[4])]
        v.append([k, c])
    json.dump(v, open(path, "w"))
variant({(768, 768): 26}, out + "/t_oproj26.json")
variant({(768, 768): 26, (768, 3072): 26}, out + "/t_oproj26_down26.json")
PY
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --steps 2000 --warmup 50 --json-out $O/ship_r$r.json > $O/ship_r$r.out 2>&1 || exit $?
  RDB_TUNE_FILE=$GRAFT_REPO_ROOT/$O/t_oproj26.json timeout -k 10 200 python3 bench.py --steps 2000 --warmup 50 --json-out $O/o26_r$r.json > $O/o26_r$r.out 2>&1 || exit $?
  RDB_TUNE_FILE=$GRAFT_REPO_ROOT/$O/t_oproj26_down26.json timeout -k 10 200 python3 bench.py --steps 2000 --warmup 50 --json-out $O/od26_r$r.json > $O/od26_r$r.out 2>&1 || exit $?
done
echo "end $(date +%T)" >> $O/progress.txt
