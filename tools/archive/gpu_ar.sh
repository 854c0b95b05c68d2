set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench/allreduce_bench.py --same-gpu --fused-norm --iters 30 > gpurun_out/ar_same_gpu.log 2>&1
