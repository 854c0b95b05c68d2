#!/bin/bash
# Round 6: hardware-queue count vs compute streams on the BERT headline (same box, interleaved).
# GPU_MAX_HW_QUEUES (HIP's default 4): with 3 compute streams + the copy stream + the null
# stream, two streams would share a hardware queue.
set -o pipefail
O=gpurun_out/r6d
mkdir -p $O
run() {  # name, env..., -- bench args
  local n=$1; shift
  timeout -k 10 300 env "$@" > $O/$n.log 2>&1 || return 1
}
for rep in 1 2; do
  run cs2_q4_$rep python bench.py --steps 200 --warmup 20 --json-out $O/cs2_q4_$rep.json || exit 1
  run cs2_q8_$rep GPU_MAX_HW_QUEUES=8 python bench.py --steps 200 --warmup 20 --json-out $O/cs2_q8_$rep.json || exit 1
  run cs3_q8_$rep GPU_MAX_HW_QUEUES=8 python bench.py --steps 200 --warmup 20 --compute-streams 3 --pipeline-depth 6 \
      --concurrency 128 --json-out $O/cs3_q8_$rep.json || exit 1
  run cs3_q4_$rep python bench.py --steps 200 --warmup 20 --compute-streams 3 --pipeline-depth 6 \
      --concurrency 128 --json-out $O/cs3_q4_$rep.json || exit 1
done
echo "exit 0"
