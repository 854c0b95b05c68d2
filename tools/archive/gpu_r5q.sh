set -o pipefail
# Round 5: BERT operating points: compute streams x pipeline depth x closed-loop
# concurrency (throughput vs p99), --steps 2000.
bash tools/fresh.sh || exit 9
O=gpurun_out/r5q
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for cfg in "2 4 96" "2 6 128" "3 6 128" "3 8 160" "2 4 96" "4 8 160"; do
  set -- $cfg
  timeout -k 10 200 python3 bench.py --steps 2000 --warmup 50 --compute-streams $1 --pipeline-depth $2 --concurrency $3 --json-out $O/cs$1_d$2_c$3_$RANDOM.json > /dev/null 2>&1 || exit $?
done
