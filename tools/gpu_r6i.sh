#!/bin/bash
# Round 6: segment stamps of the persistent halo convs (diagnostic build).
set -o pipefail
O=gpurun_out/r6i
mkdir -p $O
(cd bench/gemm_lab && hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../ray_dynamic_batching_amd/ops/csrc -DRDB_HALO_STAMPS halo_lab.hip -o /tmp/halo_lab) || exit 1
for a in "8 32 56 64 64" "6 32 56 64 64" "7 32 28 128 128"; do
  timeout -k 10 60 /tmp/halo_lab $a >> $O/stamps6.jsonl || exit 1
done
cat $O/stamps6.jsonl
