#!/bin/bash
# Round 6: halo-tile 3x3 conv -- numerics vs fp32 torch, then launch timings vs the shipped table's tiles.
set -o pipefail
O=gpurun_out/r6g
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "halo" \
    > $O/pytest_halo.log 2>&1 || { tail -30 $O/pytest_halo.log; exit 1; }
tail -3 $O/pytest_halo.log
timeout -k 10 300 python bench/conv_halo_bench.py --json-out $O/conv_halo_bench.json > $O/conv_halo_bench.log 2>&1 || { tail -20 $O/conv_halo_bench.log; exit 1; }
cat $O/conv_halo_bench.log
