# round 4: same-box A/B of the LayerNorm grid cap (RDB_LN_BLOCKS: grid-stride LN on fewer blocks so the
# other compute stream's GEMM keeps CUs) on the headline bench
set -o pipefail
rm -f gpurun_out/abe/summary.txt
bash tools/gpu_ab_env.sh 3 "RDB_AB=0" "RDB_LN_BLOCKS=128" "RDB_LN_BLOCKS=64" || exit $?
mkdir -p gpurun_out/r4q && cp gpurun_out/abe/summary.txt gpurun_out/r4q/ln_blocks_ab.txt
