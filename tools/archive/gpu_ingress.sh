# Ingress-capacity rehearsal: 8 ranks of native echo replicas (no GPU use) with the
# rank-0 load generator, at 900 us per 32-batch (~284k req/s target), 4 and 8 ingress
# threads; then the driver's short headline invocation (steps 20 / warmup 5) on the GPU.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for g in 4 8; do
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port 2961$g bench.py --gpus 8 --steps 300 --warmup 30 --backend echo --echo-service-us 900 \
    --ingress-threads $g --json-out gpurun_out/echo8_g$g.json > gpurun_out/echo8_g$g.log 2>&1 || exit 1
done
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --json-out gpurun_out/bench_s20_$i.json > gpurun_out/bench_s20_$i.log 2>&1 || exit 1
done
