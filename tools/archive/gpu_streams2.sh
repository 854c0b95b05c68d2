# Compute-stream / pipeline-depth sweep with the round-2 kernel set (fused QKV+attention),
# each config tuned in context for its own stream count, 2 rounds interleaved.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for cfg in "2 4" "3 6" "2 6" "4 8"; do
    set -- $cfg
    timeout -k 10 200 python -u bench.py --steps 600 --warmup 30 --compute-streams $1 --pipeline-depth $2 \
      --json-out gpurun_out/cs_${1}_${2}_$r.json > gpurun_out/cs_${1}_${2}_$r.log 2>&1 || exit 1
  done
done
