set -o pipefail
# Round 5: HIP runtime knobs for the graph-replay path (kernel arguments in device
# memory), interleaved A/B at --steps 2000.
bash tools/fresh.sh || exit 9
O=gpurun_out/r5n
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --steps 2000 --warmup 50 --json-out $O/base_r$r.json > $O/base_r$r.out 2>&1 || exit $?
  HIP_FORCE_DEV_KERNARG=1 timeout -k 10 200 python3 bench.py --steps 2000 --warmup 50 --json-out $O/devk_r$r.json > $O/devk_r$r.out 2>&1 || exit $?
done
for r in 1 2; do
  timeout -k 10 300 python3 bench/serve_bench.py --model resnet50 --closed 96 --seconds 8 --json-out $O/rn_base_r$r.json > $O/rn_base_r$r.out 2>&1 || exit $?
  HIP_FORCE_DEV_KERNARG=1 timeout -k 10 300 python3 bench/serve_bench.py --model resnet50 --closed 96 --seconds 8 --json-out $O/rn_devk_r$r.json > $O/rn_devk_r$r.out 2>&1 || exit $?
done
