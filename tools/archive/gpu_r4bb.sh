# round 4 final: Poisson serving curve of the headline config on the final shipped table, both batch policies
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r4bb
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for pol in timeout idle; do
  for r in 5000 10000 20000 28000 32000; do
    timeout -k 10 150 python -u bench.py --rate $r --steps 300 --warmup 30 --batch-policy $pol \
      > gpurun_out/r4bb/${pol}_$r.log 2>&1 || exit $?
  done
  timeout -k 10 150 python -u bench.py --steps 2000 --warmup 50 --batch-policy $pol > gpurun_out/r4bb/${pol}_closed.log 2>&1 || exit $?
done
