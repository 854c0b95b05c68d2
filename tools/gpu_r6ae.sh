#!/bin/bash
# Round 6: ResNet-50 bs32 single-stream graph replay, the round-3 single-stream table vs the round-6 cs1 table
# (halo 3x3 convs), interleaved x3.
set -o pipefail
O=gpurun_out/r6ae
mkdir -p $O
D=ray_dynamic_batching_amd/ops/tuned
for i in 1 2 3; do
  for t in mi355x_resnet50_B32_d2 mi355x_resnet50_B32_cs1_d2; do
    timeout -k 10 200 python -u bench/cnn_breakdown.py --model resnet50 --batch 32 --iters 100 --tune-file $D/$t.json > $O/${t}_$i.log 2>&1 || { tail -20 $O/${t}_$i.log; exit 1; }
    echo "$t $i $(tail -n 1 $O/${t}_$i.log)"
  done
done
