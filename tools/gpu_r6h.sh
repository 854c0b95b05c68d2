#!/bin/bash
# Round 6: counters of the halo-tile 3x3 conv vs the table tile on ResNet stage 1 / 2.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6h2
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES \
    --output-format csv -d $O/p1 -- python3 bench/conv_halo_bench.py --shapes 0,1 --choices halo0,halo6,halo7 --iters 3 > $O/p1.log 2>&1 || { tail -20 $O/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_UNALIGNED_STALL \
    --output-format csv -d $O/p2 -- python3 bench/conv_halo_bench.py --shapes 0,1 --choices halo0,halo6,halo7 --iters 3 > $O/p2.log 2>&1 || { tail -20 $O/p2.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -- python3 bench/conv_halo_bench.py --shapes 0,1 --choices halo0,halo6,halo7 --iters 20 > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
find $O -name "*.csv" | head -20
