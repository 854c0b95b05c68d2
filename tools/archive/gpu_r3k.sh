# full-row GEMM+LayerNorm (packed W): kernel tests + probe
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r3k
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -k "rowln" -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider -m gpu > gpurun_out/r3k/pytest.log 2>&1 || exit $?
timeout -k 10 120 python -u bench/rowln_probe.py --tune-file ray_dynamic_batching_amd/ops/tuned/mi355x_bert_L12_S128_B32_cs2_d4.json > gpurun_out/r3k/probe.json 2>&1
