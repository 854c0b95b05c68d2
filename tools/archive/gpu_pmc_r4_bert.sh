set -o pipefail
# Round-4 hardware counters of one BERT-base bs32 forward with the SHIPPED MI355X tile
# table (graph replay): one rocprofv3 pass per counter group, then the per-kernel summary.
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/pmc4b
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
cp ray_dynamic_batching_amd/ops/tuned/mi355x_bert_L12_S128_B32_cs2_d4.json gpurun_out/pmc4b/tiles.json
T=gpurun_out/pmc4b/tiles.json
B="python3 bench/bert_breakdown.py --batch 32 --iters 5 --tune-file $T"
SQ="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE"
timeout -s KILL 240 rocprofv3 --pmc $SQ --output-format csv -d gpurun_out/pmc4b/sq -o p -- $B > gpurun_out/pmc4b/sq.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc4b/fetch -o p -- $B > gpurun_out/pmc4b/fetch.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc4b/write -o p -- $B > gpurun_out/pmc4b/write.log 2>&1 && \
python3 bench/pmc_summary.py gpurun_out/pmc4b/sq gpurun_out/pmc4b/fetch gpurun_out/pmc4b/write -o gpurun_out/pmc4b/pmc_bert_forward_r4.json \
  --marker embed16_kernel --forwards 10 --top 40 --note "BERT-base bs32 seq128 forward, shipped MI355X tile table (round 4), graph replay, one counter pass per group" > gpurun_out/pmc4b/summary.log 2>&1
rc=$?
find gpurun_out/pmc4b -name "*.csv" -size +2M -delete
exit $rc
