# embed16 + key_ids: ops tests, then an env A/B of the embedding kernel form (shipped table), 3 rounds
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r3f
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_ops_gpu.py -k "embed or qkv_attention" > gpurun_out/r3f/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r3f/status.txt
case $rc in 0) ;; *) exit $rc;; esac
for r in 1 2 3; do
  for arm in "RDB_EMBED16=0" "RDB_EMBED16=1"; do
    timeout -k 10 150 env $arm python -u bench.py --steps 2000 --warmup 50 > gpurun_out/r3f/${arm}_r$r.log 2>&1
    rc=$?
    echo "$arm r$r rc=$rc $(tail -n 1 gpurun_out/r3f/${arm}_r$r.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["p99_ms"])' 2>/dev/null)" >> gpurun_out/r3f/summary.txt
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
