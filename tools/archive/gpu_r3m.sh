# Round-3 serving curve (Poisson open loop, shipped tables) + 2- and 4-rank protocol rehearsal with real engines on one GPU
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r3m
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 10000 20000 25000 28000 30000 32000; do
  timeout -k 10 150 python -u bench.py --rate $r --steps 600 --warmup 30 --json-out gpurun_out/r3m/rate_$r.json > gpurun_out/r3m/rate_$r.log 2>&1 || exit $?
done
timeout -k 10 150 python -u bench.py --steps 1000 --warmup 30 --json-out gpurun_out/r3m/closed.json > gpurun_out/r3m/closed.log 2>&1 || exit $?
for n in 2 4; do
  timeout -k 10 240 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29700 + n)) bench.py --gpus $n --steps 100 --warmup 10 --rehearse-one-gpu \
    --json-out gpurun_out/r3m/rehearse_$n.json > gpurun_out/r3m/rehearse_$n.log 2>&1 || exit $?
done
exit 0
