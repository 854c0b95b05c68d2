#!/bin/bash
# Round 6, first GPU pass: smoke, the new GPU tests (multi-GPU tier rehearsals,
# native TP leader/follower, Serve-deployed engine), driver-shaped bench, and the
# Serve-deployed BERT replica vs the direct EngineRunner on the same box.
set -o pipefail
O=gpurun_out/r6a
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_multigpu_gpu.py tests/test_models2_gpu.py > $O/pytest.log 2>&1 &&
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out $O/bench.json > $O/bench.log 2>&1 &&
timeout -k 10 400 python bench/serve_bench.py --model bert-base --closed 96 --seconds 5 \
    --json-out $O/direct.json > $O/direct.log 2>&1 &&
timeout -k 10 500 python bench/serve_bench.py --model bert-base --closed 96 --seconds 5 --via-serve \
    --json-out $O/via_serve.json > $O/via_serve.log 2>&1 &&
timeout -k 10 400 python bench/serve_batch_slice.py --seconds 8 --concurrency 64 \
    --json-out $O/slice.json > $O/slice.log 2>&1 &&
timeout -k 10 400 python bench/serve_bench.py --model resnet50 --closed 96 --seconds 5 \
    --json-out $O/resnet_direct.json > $O/resnet_direct.log 2>&1
echo "exit $?"
