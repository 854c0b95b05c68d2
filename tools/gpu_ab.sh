# A/B on one box with a fixed GEMM tile table: run 1 tunes and saves the table,
# the following runs replay it.  Usage: bash tools/gpu_ab.sh "ENV_A" "ENV_B" [steps]
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
A="$1"; B="$2"; STEPS=${3:-600}
rm -f gpurun_out/ab_tiles.json
export RDB_TUNE_FILE=$GRAFT_REPO_ROOT/gpurun_out/ab_tiles.json
timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 > gpurun_out/ab_tune.log 2>&1 && \
for i in 1 2; do
  timeout -k 10 200 env $A python -u bench.py --steps $STEPS --warmup 30 > gpurun_out/ab_A$i.log 2>&1 || exit 1
  timeout -k 10 200 env $B python -u bench.py --steps $STEPS --warmup 30 > gpurun_out/ab_B$i.log 2>&1 || exit 1
done
for f in gpurun_out/ab_A1.log gpurun_out/ab_B1.log gpurun_out/ab_A2.log gpurun_out/ab_B2.log; do
  echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"p99_ms": [0-9.]*' $f)"
done
