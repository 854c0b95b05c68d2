set -o pipefail
# Round 5: tile choices re-ranked by CU-time measured in the UN-profiled bench
# (block-stamp build): the shipped BERT table and single-GEMM alternatives.
bash tools/fresh.sh || exit 9
O=gpurun_out/r5t
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=$GRAFT_REPO_ROOT/ray_dynamic_batching_amd/_variants/stamps/_rdb_ops.cpython-310-x86_64-linux-gnu.so
S=ray_dynamic_batching_amd/ops/tuned/mi355x_bert_L12_S128_B32_cs2_d4.json
python3 - "$S" $O <<'PY'
import json, sys
src, out = sys.argv[1], sys.argv[2]
t = json.load(open(src))
def variant(name, nk, cfg):
    v = [[k, (cfg if (k[0] == "gemm" and k[2] == 4096 and (k[3], k[4]) == nk and k[6] in ("none", "gelu")) else c)] for k, c in t]
    json.dump(v, open(f"{out}/t_{name}.json", "w"))
variant("oproj_cfg10", (768, 768), 10)      # round-3 o-proj: 4-wave 128x96, 256 blocks
variant("ffnup_cfg22", (3072, 768), 22)     # FFN-up on the 256x256 ping-pong tile
variant("ffndown_cfg9", (768, 3072), 9)     # FFN-down on the 4-wave 64x96 tile
PY
for arm in ship oproj_cfg10 ffnup_cfg22 ffndown_cfg9; do
  TF=$S; [ $arm != ship ] && TF=$GRAFT_REPO_ROOT/$O/t_$arm.json
  RDB_OPS_SO=$V RDB_TUNE_FILE=$TF timeout -k 10 300 python3 bench.py --steps 100 --warmup 50 --stamps-out $O/st_$arm.npy --json-out $O/b_$arm.json > /dev/null 2> $O/b_$arm.err || exit $?
  timeout -k 10 300 python3 bench/stamp_timeline.py $O/st_$arm.npy -o $O/tl_$arm.json > /dev/null 2>&1 || exit $?
  rm -f $O/st_$arm.npy
done
