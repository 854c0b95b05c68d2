set -o pipefail
# Round 5: vendor-kernel arms in the same native engine (BERT: hipBLASLt + SDPA
# under hipGraph capture; ResNet-50: MIOpen channels_last fp16), the
# reference-equivalent baseline, the HIP arms on the same box, and the new GPU
# tests (Serve TP group at world 8 on one GPU).
bash tools/fresh.sh || exit 9
O=gpurun_out/r5b
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_serve_tp_gpu.py > $O/pytest_tp.log 2>&1 && \
timeout -k 10 300 python3 bench.py --steps 2000 --warmup 50 --json-out $O/bench_hip_a.json > $O/bench_hip_a.out 2> $O/bench_hip_a.err && \
timeout -k 10 300 python3 bench.py --steps 2000 --warmup 50 --backend torch --json-out $O/bench_torch_a.json > $O/bench_torch_a.out 2> $O/bench_torch_a.err && \
timeout -k 10 300 python3 bench.py --steps 2000 --warmup 50 --json-out $O/bench_hip_b.json > $O/bench_hip_b.out 2> $O/bench_hip_b.err && \
timeout -k 10 300 python3 bench.py --steps 2000 --warmup 50 --backend torch --json-out $O/bench_torch_b.json > $O/bench_torch_b.out 2> $O/bench_torch_b.err && \
timeout -k 10 300 python3 bench/baseline_serve.py --json-out $O/baseline_serve.json > $O/baseline.out 2> $O/baseline.err && \
timeout -k 10 300 python3 bench/serve_bench.py --model resnet50 --closed 96 --seconds 8 --json-out $O/resnet_hip.json > $O/resnet_hip.out 2> $O/resnet_hip.err && \
timeout -k 10 300 python3 bench/serve_bench.py --model resnet50 --closed 96 --seconds 8 --backend torch --json-out $O/resnet_torch.json > $O/resnet_torch.out 2> $O/resnet_torch.err
rc=$?
exit $rc
