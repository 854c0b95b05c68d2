# Round-4 hardware counters of one ResNet-50 bs32 forward (graph replay) with a given
# tile table (arg 1): one rocprofv3 --pmc pass per counter group, then the per-kernel summary.
set -o pipefail
bash tools/fresh.sh || exit 9
T=${1:-ray_dynamic_batching_amd/ops/tuned/mi355x_resnet50_B32_d2.json}
mkdir -p gpurun_out/pmc4r
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python3 bench/cnn_breakdown.py --model resnet50 --batch 32 --iters 5 --tune-file $T"
SQ="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE"
timeout -s KILL 240 rocprofv3 --pmc $SQ --output-format csv -d gpurun_out/pmc4r/sq -o p -- $B > gpurun_out/pmc4r/sq.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc4r/fetch -o p -- $B > gpurun_out/pmc4r/fetch.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc4r/write -o p -- $B > gpurun_out/pmc4r/write.log 2>&1 && \
python3 bench/pmc_summary.py gpurun_out/pmc4r/sq gpurun_out/pmc4r/fetch gpurun_out/pmc4r/write -o gpurun_out/pmc4r/pmc_resnet50_forward_r4.json \
  --marker softmax_topk --forwards 10 --top 40 --note "ResNet-50 bs32 fp16 forward, round-4 tile table ($(basename $T)), graph replay, one counter pass per group" > gpurun_out/pmc4r/summary.log 2>&1
rc=$?
find gpurun_out/pmc4r -name "*.csv" -size +2M -delete
exit $rc
