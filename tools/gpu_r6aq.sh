#!/bin/bash
# Round 6 closing run on the final tree (halo patch swizzle included): smoke + pytest -m gpu (the driver's
# round-end tier), then the driver's bench command x5 and ResNet-50 closed loop 128 x2.
set -o pipefail
O=gpurun_out/${OUT:-r6aq}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -n 1 $O/smoke.log
timeout -k 10 1000 python -u -m pytest tests/ -q -m gpu --maxfail=5 --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/pytest_gpu.log 2>&1
rc=$?
tail -n 3 $O/pytest_gpu.log
[ $rc = 0 ] || exit $rc
for i in 1 2 3 4 5; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_$i.log 2>&1 || { tail -20 $O/drv_$i.log; exit 1; }
  grep '^{"metric"' $O/drv_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("drv", d["value"], d["p50_ms"], d["p99_ms"])'
done
for i in 1 2; do
  timeout -k 10 300 python bench/serve_bench.py --model resnet50 --closed 128 --seconds 5 --json-out $O/rn_c128_$i.json > $O/rn_c128_$i.log 2>&1 || { tail -20 $O/rn_c128_$i.log; exit 1; }
  python3 -c "import json; p=json.load(open('$O/rn_c128_$i.json'))['points'][0]; print('resnet c128', p['req_per_s'], p['p50_ms'], p['p99_ms'])"
done
