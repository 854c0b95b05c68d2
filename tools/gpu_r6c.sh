#!/bin/bash
# Round 6 GEMM lab: shipped ping-pong tiles vs the loader-wave ping-pong (bench/gemm_lab/gemm_ppl.h),
# alone and as two concurrent streams; every result checked against an fp32 reference GEMM.
set -o pipefail
O=gpurun_out/r6c
mkdir -p $O
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I ray_dynamic_batching_amd/ops/csrc \
    -include bench/gemm_lab/lab_ppl.h bench/gemm_lab/gemm_lab.hip -o /tmp/lab_ppl > $O/build.log 2>&1 &&
timeout -k 10 180 /tmp/lab_ppl --iters 50 --concurrent > $O/lab_ppl.txt 2>&1
echo "exit $?"
