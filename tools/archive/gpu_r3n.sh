# residual-free 16-bit-staged epilogue + pk-friendly GELU + tile 23: GEMM/model tests, then a 3-round bench A/B
#   old   = variant build with the f32-staged epilogue and the previous GELU (RDB_EPI_F32_STAGING, RDB_GELU_OLD)
#   new   = default build, shipped table;   new23 = default build, FFN-up on tile 23
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r3n
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -k "linear or qkv" tests/test_models_fp32_gpu.py -v --timeout 120 \
  --timeout-method thread -p no:cacheprovider -m gpu > gpurun_out/r3n/pytest.log 2>&1 || exit $?
OLD=ray_dynamic_batching_amd/_variants/epi_old/_rdb_ops.cpython-310-x86_64-linux-gnu.so
run() {  # name, RDB_OPS_SO value ("" = default), table
  RDB_OPS_SO=$2 timeout -k 10 150 python -u bench.py --steps 2000 --warmup 50 --tile-table $3 > gpurun_out/r3n/$1.log 2>&1
  rc=$?
  echo "$1 rc=$rc $(tail -n 1 gpurun_out/r3n/$1.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["p99_ms"])' 2>/dev/null)" >> gpurun_out/r3n/summary.txt
  return $rc
}
for r in 1 2 3; do
  run old_r$r $OLD tools/ab_tables_r3n/A_shipped.json || exit $?
  run new_r$r "" tools/ab_tables_r3n/A_shipped.json || exit $?
  run new23_r$r "" tools/ab_tables_r3n/B_ffn1_23.json || exit $?
done
exit 0
