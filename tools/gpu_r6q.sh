#!/bin/bash
# Round 6: GEMM lab -- per-wave tile size (LDS bytes per MFMA) on the BERT shapes.
set -o pipefail
O=gpurun_out/r6q
mkdir -p $O
(cd bench/gemm_lab && hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../ray_dynamic_batching_amd/ops/csrc -DLAB_SET_BIG gemm_lab.hip -o /tmp/gemm_lab_big) || exit 1
timeout -k 10 240 /tmp/gemm_lab_big --iters 50 --concurrent > $O/lab_big.txt 2>&1 || { tail -20 $O/lab_big.txt; exit 1; }
cat $O/lab_big.txt
