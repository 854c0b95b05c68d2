set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u bench/bert_breakdown.py --batch 32 > gpurun_out/bd_plain.log 2>&1 && \
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bd -o bd -- python3 bench/bert_breakdown.py --batch 32 --iters 50 > gpurun_out/bd_prof.log 2>&1
