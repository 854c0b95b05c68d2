set -o pipefail
# Round 5: is the driver-shaped window (--steps 20 --warmup 5) slower because of
# pipeline fill / drain or because the GPU is still warming up?  Interleaved.
bash tools/fresh.sh || exit 9
O=gpurun_out/r5l
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --json-out $O/w5_r$r.json > $O/w5_r$r.out 2>&1 || exit $?
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 300 --json-out $O/w300_r$r.json > $O/w300_r$r.out 2>&1 || exit $?
  timeout -k 10 200 python3 bench.py --steps 300 --warmup 5 --json-out $O/s300_r$r.json > $O/s300_r$r.out 2>&1 || exit $?
done
