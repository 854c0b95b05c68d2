# Ingress A/B at 8 ranks with native echo replicas (CPU only, 900 us per 32-batch),
# then the 2-rank protocol with real engines on one GPU (per-rank ingress).
set -o pipefail
mkdir -p gpurun_out/ingress
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
nproc > gpurun_out/ingress/nproc.txt; python -c "import os; print(len(os.sched_getaffinity(0)))" >> gpurun_out/ingress/nproc.txt
P=29600
for i in 1 2; do for mode in per-rank rank0; do
  P=$((P+1))
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port $P \
    bench.py --gpus 8 --steps 300 --warmup 20 --backend echo --echo-service-us 900 --ingress $mode \
    > gpurun_out/ingress/echo8_${mode}_$i.log 2>&1 || exit 1
done; done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29650 \
  bench.py --gpus 2 --steps 100 --warmup 10 --rehearse-one-gpu > gpurun_out/ingress/rehearse2.log 2>&1 || exit 1
grep -h '^{' gpurun_out/ingress/*.log | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['n_gpus'], d['ingress'], d['value'], d['p99_ms'])"
