# round 4: staged-LN (partial statistics) numerics + spill-fix numerics, then same-box A/B:
# shipped vs LN-in-GEMM (pstats) vs FFN-up 256x256 / 256x192 tiles (now spill-free)
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r4f
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ln_staged_gpu.py tests/test_ops_gpu.py tests/test_models_gpu.py > gpurun_out/r4f/pytest.log 2>&1 || exit $?
rm -f gpurun_out/abe/summary.txt
bash tools/gpu_ab_env.sh 3 "RDB_AB=0" "RDB_BERT_LN_PSTATS=1" "RDB_AB=0 -- --tile-table tools/ab_tables_r4/B_ffn1_22.json" "RDB_AB=0 -- --tile-table tools/ab_tables_r4/C_ffn1_24.json" "RDB_BERT_LN_PSTATS=1 -- --tile-table tools/ab_tables_r4/C_ffn1_24.json"
