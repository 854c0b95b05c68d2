# round 4: ResNet-50 serving curve + PMC table with the shipped cs2/d4 table, then the
# staged-LayerNorm numerics and a same-box BERT A/B: shipped vs LayerNorm folded into
# the GEMMs with partial statistics (RDB_BERT_LN_PSTATS=1), with / without FFN-up on cfg 24
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r4k
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u bench/serve_bench.py --model resnet50 --closed 96 --seconds 4 \
  --rates 2000,4000,8000,12000,16000,20000,24000,28000,32000 --json-out gpurun_out/r4k/resnet50_serving_r4.json \
  > gpurun_out/r4k/resnet_curve.log 2>&1 || exit $?
bash tools/gpu_pmc_r4_resnet.sh ray_dynamic_batching_amd/ops/tuned/mi355x_resnet50_B32_cs2_d4.json || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ln_staged_gpu.py \
  > gpurun_out/r4k/pytest_ln_staged.log 2>&1 || exit $?
rm -f gpurun_out/abe/summary.txt
bash tools/gpu_ab_env.sh 2 "RDB_AB=0" "RDB_BERT_LN_PSTATS=1" "RDB_BERT_LN_PSTATS=1 -- --tile-table tools/ab_tables_r4/C_ffn1_24.json"
