# new skinny kernel: tests + isolated timing; then headline A/B of in-kernel key lengths (RDB_BERT_KEY_IDS)
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r3g
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_models_gpu.py -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider -m gpu > gpurun_out/r3g/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r3g/status.txt
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 120 python -u bench/skinny_probe.py --json gpurun_out/r3g/skinny_new.json > gpurun_out/r3g/skinny.log 2>&1 || exit $?
for r in 1 2 3; do
  for arm in "RDB_BERT_KEY_IDS=0" "RDB_BERT_KEY_IDS=1"; do
    timeout -k 10 150 env $arm python -u bench.py --steps 2000 --warmup 50 > gpurun_out/r3g/${arm}_r$r.log 2>&1
    rc=$?
    echo "$arm r$r rc=$rc $(tail -n 1 gpurun_out/r3g/${arm}_r$r.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["p99_ms"])' 2>/dev/null)" >> gpurun_out/r3g/summary.txt
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
