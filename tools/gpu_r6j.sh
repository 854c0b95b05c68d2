#!/bin/bash
# Round 6: register-weight halo conv -- numerics, timings, stamps-free.
set -o pipefail
O=gpurun_out/r6j3
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "halo" \
    > $O/pytest_halo.log 2>&1 || { tail -30 $O/pytest_halo.log; exit 1; }
tail -2 $O/pytest_halo.log
timeout -k 10 300 python bench/conv_halo_bench.py --json-out $O/conv_halo_bench.json --shapes 2,3 > $O/conv_halo_bench.log 2>&1 || { tail -20 $O/conv_halo_bench.log; exit 1; }
grep shape $O/conv_halo_bench.log | cut -c1-170
