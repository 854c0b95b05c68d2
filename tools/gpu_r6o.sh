#!/bin/bash
# Round 6: kernel-trace stats of the final tree: BERT headline (bench.py) and ResNet-50 serving.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6o
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bert -- python3 bench.py --steps 100 --warmup 10 \
    --json-out $O/bert_bench.json > $O/bert.log 2>&1 || { tail -5 $O/bert.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/resnet -- python3 bench/serve_bench.py --model resnet50 \
    --closed 96 --seconds 3 --json-out $O/resnet_bench.json > $O/resnet.log 2>&1 || { tail -5 $O/resnet.log; exit 1; }
find $O -name "*kernel_stats.csv"
