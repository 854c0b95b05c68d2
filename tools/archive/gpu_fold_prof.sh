set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fp_on -o p -- python3 bench/bert_breakdown.py --batch 32 --iters 50 --tune-file gpurun_out/fp_tune_on.json > gpurun_out/fp_on.log 2>&1 && \
RDB_BERT_FOLD_LN=0 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fp_off -o p -- python3 bench/bert_breakdown.py --batch 32 --iters 50 --tune-file gpurun_out/fp_tune_off.json > gpurun_out/fp_off.log 2>&1
