# fused-attention key_ids tests + BERT model tests, then the bench profile (shipped table)
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r3e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_ops_gpu.py tests/test_models_gpu.py tests/test_models_fp32_gpu.py \
  > gpurun_out/r3e/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r3e/status.txt
case $rc in 0) ;; *) exit $rc;; esac
bash tools/gpu_prof_r3.sh; rc=$?; echo "prof rc=$rc" >> gpurun_out/r3e/status.txt
exit $rc
