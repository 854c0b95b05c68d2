set -o pipefail
# Round 5: hardware counters of hipBLASLt vs our GEMM kernels on the BERT shapes
# and 4096^3 (bench/gemm_vendor_probe.py), one rocprofv3 --pmc pass per group.
bash tools/fresh.sh || exit 9
O=gpurun_out/pmc5g
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python3 bench/gemm_vendor_probe.py --iters 20 --reps 2"
SQ="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE"
timeout -s KILL 300 rocprofv3 --pmc $SQ --output-format csv -d $O/sq -o p -- $B > $O/sq.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $O/fetch -o p -- $B > $O/fetch.log 2>&1 && \
python3 bench/pmc_summary.py $O/sq $O/fetch -o $O/pmc_gemm_side_by_side_r5.json --top 40 \
  --note "hipBLASLt (torch F.linear / _addmm_activation) vs this repo's shipped BERT tiles, standalone graph replays, bench/gemm_vendor_probe.py; one counter pass per group" > $O/summary.log 2>&1
rc=$?
find $O -name "*.csv" -size +2M -delete
exit $rc
