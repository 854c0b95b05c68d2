# N-rank bench protocol rehearsal with real engines on ONE GPU (per-rank ingress, gloo): 4 and 8 ranks
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r3w
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for n in 4 8; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29700+n)) \
    bench.py --gpus $n --steps 40 --warmup 5 --rehearse-one-gpu > gpurun_out/r3w/rehearse$n.log 2>&1 || exit $?
done
grep -h '^{' gpurun_out/r3w/*.log > gpurun_out/r3w/lines.jsonl
