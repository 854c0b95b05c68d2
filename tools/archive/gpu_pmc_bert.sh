set -o pipefail
# Hardware counters of every kernel of one BERT-base bs32 forward (graph replay):
# one rocprofv3 pass per counter group (SQ, FETCH, WRITE), then the summary.
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -f gpurun_out/pmc_tune.json
# tile tuning runs once WITHOUT counters (under --pmc every dispatch is serialised and
# the tuning sweep alone outlasts the pass limit); the counter passes replay the table
timeout -k 10 200 python3 bench/bert_breakdown.py --batch 32 --iters 2 --tune-file gpurun_out/pmc_tune.json > gpurun_out/pmc_tune.log 2>&1 && \
SQ="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE"
timeout -s KILL 240 rocprofv3 --pmc $SQ --output-format csv -d gpurun_out/pmc_sq -o p -- python3 bench/bert_breakdown.py --batch 32 --iters 5 --tune-file gpurun_out/pmc_tune.json > gpurun_out/pmc_sq.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_fetch -o p -- python3 bench/bert_breakdown.py --batch 32 --iters 5 --tune-file gpurun_out/pmc_tune.json > gpurun_out/pmc_fetch.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_write -o p -- python3 bench/bert_breakdown.py --batch 32 --iters 5 --tune-file gpurun_out/pmc_tune.json > gpurun_out/pmc_write.log 2>&1 && \
python3 bench/pmc_summary.py gpurun_out/pmc_sq gpurun_out/pmc_fetch gpurun_out/pmc_write -o gpurun_out/pmc_bert_forward.json \
  --marker seq_lens_kernel --forwards 10 --top 40 --note "BERT-base bs32 seq128 forward (eager warmup + graph replay), one counter pass per group" > gpurun_out/pmc_summary.log 2>&1
