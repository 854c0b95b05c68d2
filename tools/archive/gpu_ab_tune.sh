# A/B where each arm tunes its own tiles (no fixed table): alternating runs.
# Usage: bash tools/gpu_ab_tune.sh "ENV_A" "ENV_B" [steps] [rounds]
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
A="$1"; B="$2"; STEPS=${3:-1000}; R=${4:-2}
for i in $(seq 1 $R); do
  timeout -k 10 240 env $A python -u bench.py --steps $STEPS --warmup 30 > gpurun_out/abt_A$i.log 2>&1 || exit 1
  timeout -k 10 240 env $B python -u bench.py --steps $STEPS --warmup 30 > gpurun_out/abt_B$i.log 2>&1 || exit 1
done
for f in gpurun_out/abt_A*.log gpurun_out/abt_B*.log; do
  echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"p99_ms": [0-9.]*' $f) $(grep -o 'in_context_tile_changes.*' $f | head -c 150)"
done
