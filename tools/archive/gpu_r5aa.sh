set -o pipefail
# Round 5: fused QKV + attention variant at bs32 in the engine: shipped cfg 1
# (8 waves, 2 stages, 2 blocks / CU) vs cfg 4 (two sequences per block) vs cfg 3.
bash tools/fresh.sh || exit 9
O=gpurun_out/r5aa
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
S=ray_dynamic_batching_amd/ops/tuned/mi355x_bert_L12_S128_B32_cs2_d4.json
python3 - "$S" $O <<'PY'
import json, sys
src, out = sys.argv[1], sys.argv[2]
t = json.load(open(src))
for cfg in (3, 4):
    v = [[k, (cfg if (k[0] == "qkv_attn" and k[2] == 32) else c)] for k, c in t]
    json.dump(v, open(f"{out}/t_qa{cfg}.json", "w"))
PY
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --steps 2000 --warmup 50 --json-out $O/ship_r$r.json > /dev/null 2>&1 || exit $?
  RDB_TUNE_FILE=$GRAFT_REPO_ROOT/$O/t_qa4.json timeout -k 10 200 python3 bench.py --steps 2000 --warmup 50 --json-out $O/qa4_r$r.json > /dev/null 2>&1 || exit $?
  RDB_TUNE_FILE=$GRAFT_REPO_ROOT/$O/t_qa3.json timeout -k 10 200 python3 bench.py --steps 2000 --warmup 50 --json-out $O/qa3_r$r.json > /dev/null 2>&1 || exit $?
done
