# Single-stream forward kernel traces of two model settings (bench/bert_breakdown.py).
# Usage: bash tools/gpu_prof2.sh "ENV_A" "ENV_B"
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
i=0
for e in "$1" "$2"; do
  i=$((i+1))
  timeout -k 10 180 env $e rocprofv3 --kernel-trace --output-format csv -d gpurun_out/p2_$i -o p -- python3 bench/bert_breakdown.py --batch 32 --iters 50 > gpurun_out/p2_$i.log 2>&1 || exit 1
done
