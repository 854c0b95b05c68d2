#!/bin/bash
# Round 6: the driver's round-end GPU tier on this tree (cs3/d6 defaults, halo convs): smoke + pytest -m gpu.
set -o pipefail
O=gpurun_out/r6w
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 1050 python -u -m pytest tests/ -q -m gpu --maxfail=5 --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/pytest_gpu.log 2>&1
rc=$?
tail -15 $O/pytest_gpu.log
exit $rc
