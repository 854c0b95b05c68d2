#!/bin/bash
# Round 6: stride-2 halo convs -- numerics, then graph-replayed layer timings (stride 1 and 2) vs the shipped table.
set -o pipefail
O=gpurun_out/r6t
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py -k "halo" \
    > $O/pytest_halo.log 2>&1 || { tail -30 $O/pytest_halo.log; exit 1; }
tail -1 $O/pytest_halo.log
timeout -k 10 400 python bench/conv_halo_bench.py --stride 2 --iters 20 --json-out $O/s2.json > $O/s2.log 2>&1 || { tail -20 $O/s2.log; exit 1; }
timeout -k 10 400 python bench/conv_halo_bench.py --stride 1 --iters 20 --json-out $O/s1.json > $O/s1.log 2>&1 || { tail -20 $O/s1.log; exit 1; }
grep shape $O/s2.log $O/s1.log | sed 's/gpurun_out.r6t.//' | cut -c1-175
