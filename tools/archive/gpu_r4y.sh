# round 4: config 3 (BERT dyn-batch <= 16): FFN-down at bs16 on the 96/48-block ping-pong tiles (CU-time) vs shipped
set -o pipefail
rm -f gpurun_out/abt/summary.txt
AB_TABLES=tools/ab_tables_r4y bash tools/gpu_ab_tables.sh 2 --max-batch 16 || exit $?
mkdir -p gpurun_out/r4y && cp gpurun_out/abt/summary.txt gpurun_out/r4y/tables_ab_b16.txt
