mkdir -p gpurun_out
for cs in 2 3 4 2 3 4; do
  timeout -k 10 150 python -u bench.py --steps 3000 --compute-streams $cs --pipeline-depth $((cs>4?cs:4)) > gpurun_out/cs_$cs.log 2>&1 || exit 1
  grep -h '^{"metric' gpurun_out/cs_$cs.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print($cs, d['value'], d['p50_ms'], d['p99_ms'])" >> gpurun_out/cs_summary.txt
done
