set -o pipefail
# Round 5: FFN-up tile at bs32 after the grouped walk: shipped (cfg 23) vs cfg 22 / cfg 25, interleaved.
bash tools/fresh.sh || exit 9
O=gpurun_out/r5y
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
S=ray_dynamic_batching_amd/ops/tuned/mi355x_bert_L12_S128_B32_cs2_d4.json
python3 - "$S" $O <<'PY'
import json, sys
src, out = sys.argv[1], sys.argv[2]
t = json.load(open(src))
for cfg in (22, 25):
    v = [[k, (cfg if (k[0] == "gemm" and k[2] == 4096 and (k[3], k[4]) == (3072, 768)) else c)] for k, c in t]
    json.dump(v, open(f"{out}/t_up{cfg}.json", "w"))
PY
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --steps 2000 --warmup 50 --json-out $O/ship_r$r.json > /dev/null 2>&1 || exit $?
  RDB_TUNE_FILE=$GRAFT_REPO_ROOT/$O/t_up22.json timeout -k 10 200 python3 bench.py --steps 2000 --warmup 50 --json-out $O/up22_r$r.json > /dev/null 2>&1 || exit $?
  RDB_TUNE_FILE=$GRAFT_REPO_ROOT/$O/t_up25.json timeout -k 10 200 python3 bench.py --steps 2000 --warmup 50 --json-out $O/up25_r$r.json > /dev/null 2>&1 || exit $?
done
