# fused QKV+attention at 80 KiB (two blocks per CU for cfgs 1/3): kernel tests, then bench A/Bs
#   bs32: shipped (cfg 4) vs cfg 3 vs cfg 1 (3 rounds); bs16: shipped vs FFN-up on tile 23 (2 rounds)
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r3o
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -k "qkv or attention" -v --timeout 120 \
  --timeout-method thread -p no:cacheprovider -m gpu > gpurun_out/r3o/pytest.log 2>&1 || exit $?
run() {  # name, table, extra args
  timeout -k 10 150 python -u bench.py --steps 2000 --warmup 50 --tile-table $2 $3 > gpurun_out/r3o/$1.log 2>&1
  rc=$?
  echo "$1 rc=$rc $(tail -n 1 gpurun_out/r3o/$1.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["p99_ms"])' 2>/dev/null)" >> gpurun_out/r3o/summary.txt
  return $rc
}
for r in 1 2 3; do
  for t in A_shipped B_qkv3 C_qkv1; do run ${t}_r$r tools/ab_tables_r3o/$t.json "" || exit $?; done
done
for r in 1 2; do
  for t in b16_A_shipped b16_B_ffn1_23; do run ${t}_r$r tools/ab_tables_r3o/$t.json "--max-batch 16" || exit $?; done
done
exit 0
