set -o pipefail
# Round 5: ResNet-50 3x3 convolutions moved to the ping-pong conv tiles chosen by
# CU-time (fewer blocks, the other compute stream fills the CUs) vs the shipped
# table, interleaved closed-loop runs.
bash tools/fresh.sh || exit 9
O=gpurun_out/r5v
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
S=ray_dynamic_batching_amd/ops/tuned/mi355x_resnet50_B32_cs2_d4.json
python3 - "$S" $O <<'PY'
import json, sys
src, out = sys.argv[1], sys.argv[2]
t = json.load(open(src))
PP = 1 << 17
def variant(name, changes):
    v = []
    for k, c in t:
        if k[0] == "conv" and k[1] == 32 and tuple(k[2:10]) in changes:
            c = changes[tuple(k[2:10])]
        v.append([k, c])
    json.dump(v, open(f"{out}/t_{name}.json", "w"))
s23 = {(56, 56, 128, 128, 3, 3, 2, 1): PP | 0, (28, 28, 128, 128, 3, 3, 1, 1): PP | 0,
       (28, 28, 256, 256, 3, 3, 2, 1): PP | 1 | (2 << 8), (14, 14, 256, 256, 3, 3, 1, 1): PP | 1 | (2 << 8)}
s4 = {(14, 14, 512, 512, 3, 3, 2, 1): PP | 1 | (4 << 8), (7, 7, 512, 512, 3, 3, 1, 1): PP | 1 | (4 << 8)}
variant("pp23", s23)
variant("pp234", {**s23, **s4})
PY
for r in 1 2 3; do
  for arm in ship pp23 pp234; do
    TF=$S; [ $arm != ship ] && TF=$GRAFT_REPO_ROOT/$O/t_$arm.json
    RDB_TUNE_FILE=$TF timeout -k 10 300 python3 bench/serve_bench.py --model resnet50 --closed 96 --seconds 8 --json-out $O/${arm}_r$r.json > $O/${arm}_r$r.out 2>&1 || exit $?
  done
done
