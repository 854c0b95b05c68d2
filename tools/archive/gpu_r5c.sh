set -o pipefail
# Round 5: the 4-wave big-wave-tile GEMM lab, then the rest of the r5b arms
# (reference-equivalent baseline, ResNet-50 HIP vs MIOpen in the same engine).
bash tools/fresh.sh || exit 9
O=gpurun_out/r5c
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 ./labbin/w4_lab --iters 50 --concurrent > $O/w4_lab.txt 2>&1 && \
timeout -k 10 300 python3 bench/baseline_serve.py --json-out $O/baseline_serve.json > $O/baseline.out 2> $O/baseline.err && \
timeout -k 10 300 python3 bench/serve_bench.py --model resnet50 --closed 96 --seconds 8 --json-out $O/resnet_hip.json > $O/resnet_hip.out 2> $O/resnet_hip.err && \
timeout -k 10 300 python3 bench/serve_bench.py --model resnet50 --closed 96 --seconds 8 --backend torch --json-out $O/resnet_torch.json > $O/resnet_torch.out 2> $O/resnet_torch.err
