set -o pipefail
# Round 5: multi-rank rehearsal of bench.py (N ranks on one GPU, gloo; not a
# measurement) after the NUMA / deferred-ring changes, and ResNet-50 engine
# configurations (compute streams x closed-loop depth).
bash tools/fresh.sh || exit 9
O=gpurun_out/r5k
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 bench.py --gpus 2 --rehearse-one-gpu --steps 50 --warmup 10 > $O/rehearse2.out 2> $O/rehearse2.err && \
timeout -k 10 300 python3 bench.py --gpus 4 --rehearse-one-gpu --steps 50 --warmup 10 > $O/rehearse4.out 2> $O/rehearse4.err || exit $?
for cfg in "2 4 96" "3 6 128" "2 6 128" "3 6 96"; do
  set -- $cfg
  timeout -k 10 300 python3 bench/serve_bench.py --model resnet50 --compute-streams $1 --pipeline-depth $2 --closed $3 --seconds 8 --json-out $O/resnet_cs$1_d$2_c$3.json > $O/resnet_cs$1_d$2_c$3.out 2>&1 || exit $?
done
