# round 4: same-box tile-table A/B on the headline bench: o-proj on 64x96 (cfg 9, fastest alone),
# FFN-down on 64x64 (cfg 3, fastest alone), FFN-up on the 256x192 ping-pong tile (cfg 25, fastest alone)
set -o pipefail
rm -f gpurun_out/abt/summary.txt
AB_TABLES=tools/ab_tables_r4s bash tools/gpu_ab_tables.sh 3 || exit $?
mkdir -p gpurun_out/r4s && cp gpurun_out/abt/summary.txt gpurun_out/r4s/tables_ab.txt
