# two-sequence fused attention: kernel tests, then a 4-round tile-table A/B (shipped vs qkv cfg 4)
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r3h
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -k "qkv" tests/test_models_gpu.py -v --timeout 120 \
  --timeout-method thread -p no:cacheprovider -m gpu > gpurun_out/r3h/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r3h/status.txt
case $rc in 0) ;; *) exit $rc;; esac
for r in 1 2 3 4; do
  for t in tools/ab_tables/*.json; do
    n=$(basename $t .json)
    timeout -k 10 150 python -u bench.py --steps 2000 --warmup 50 --tile-table $t > gpurun_out/r3h/${n}_r$r.log 2>&1
    rc=$?
    echo "$n r$r rc=$rc $(tail -n 1 gpurun_out/r3h/${n}_r$r.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["p99_ms"])' 2>/dev/null)" >> gpurun_out/r3h/summary.txt
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
