set -o pipefail
# Round 5: improved 4-wave GEMM lab (standalone + 2-stream), ResNet-50 HIP vs
# MIOpen (channels_last fp16, weights converted once) in the same engine.
bash tools/fresh.sh || exit 9
O=gpurun_out/r5d
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 ./labbin/w4_lab --iters 50 > $O/w4_lab.txt 2>&1 && \
timeout -k 10 240 ./labbin/w4_lab --iters 50 --concurrent > $O/w4_lab_conc.txt 2>&1 && \
timeout -k 10 300 python3 bench/serve_bench.py --model resnet50 --closed 96 --seconds 8 --json-out $O/resnet_hip.json > $O/resnet_hip.out 2> $O/resnet_hip.err && \
timeout -k 10 300 python3 bench/serve_bench.py --model resnet50 --closed 96 --seconds 8 --backend torch --json-out $O/resnet_torch.json > $O/resnet_torch.out 2> $O/resnet_torch.err
