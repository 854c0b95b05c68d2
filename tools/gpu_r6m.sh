#!/bin/bash
# Round 6: PMC counters of the halo convs on the real (stamp-free) kernels via the lab harness.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6m
mkdir -p $O
(cd bench/gemm_lab && hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../ray_dynamic_batching_amd/ops/csrc halo_lab.hip -o /tmp/halo_lab_real) || exit 1
for a in "12 32 56 64 64" "0 32 56 64 64"; do
  n=$(echo $a | cut -d' ' -f1)
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES \
      --output-format csv -d $O/v$n -- /tmp/halo_lab_real $a > $O/v$n.log 2>&1 || { tail -5 $O/v$n.log; exit 1; }
  timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_VALU SQ_INSTS_MFMA \
      --output-format csv -d $O/w$n -- /tmp/halo_lab_real $a > $O/w$n.log 2>&1 || { tail -5 $O/w$n.log; exit 1; }
done
find $O -name "*counter_collection.csv"
