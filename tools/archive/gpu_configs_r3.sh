# Round-3 evidence for BASELINE configs 2 / 3 / 4: TP=8 tests on one GPU, BERT bs16 and ResNet-50 bs32
# tile tables, the ResNet-50 Poisson serving curve, and the conv kernels' counters.
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/cfg
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests/test_tp8_gpu.py -x -v --timeout 600 --timeout-method thread -p no:cacheprovider -s -k "llama or replica" > gpurun_out/cfg/tp8.log 2>&1
echo "tp8 rc=$?" >> gpurun_out/cfg/status.txt
rm -f gpurun_out/cfg/tt_b16.json gpurun_out/cfg/tt_resnet50.json
timeout -k 10 240 env RDB_TUNE_FILE=$GRAFT_REPO_ROOT/gpurun_out/cfg/tt_b16.json python -u bench.py --max-batch 16 --steps 300 --warmup 30 --tile-table none \
  --json-out gpurun_out/cfg/bench_b16_tune.json > gpurun_out/cfg/bench_b16_tune.log 2>&1 && \
timeout -k 10 240 env RDB_TUNE_FILE=$GRAFT_REPO_ROOT/gpurun_out/cfg/tt_b16.json python -u bench.py --max-batch 16 --steps 600 --warmup 30 \
  --json-out gpurun_out/cfg/bench_b16_replay.json > gpurun_out/cfg/bench_b16_replay.log 2>&1 && \
echo "b16 ok" >> gpurun_out/cfg/status.txt && \
timeout -k 10 200 python -u bench/cnn_breakdown.py --model resnet50 --batch 32 --iters 50 --tune-file gpurun_out/cfg/tt_resnet50.json > gpurun_out/cfg/resnet_bd.log 2>&1 && \
timeout -k 10 400 env RDB_TUNE_FILE=$GRAFT_REPO_ROOT/gpurun_out/cfg/tt_resnet50.json python -u bench/serve_bench.py --model resnet50 --rates 2000,4000,8000,12000,16000,20000 \
  --closed 96 --seconds 4 --json-out gpurun_out/cfg/resnet50_serving_r3.json > gpurun_out/cfg/resnet50_serving.log 2>&1 && \
echo "resnet serving ok" >> gpurun_out/cfg/status.txt && \
SQ="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE" && \
timeout -s KILL 240 rocprofv3 --pmc $SQ --output-format csv -d gpurun_out/cfg/pmc_sq -o p -- python3 bench/cnn_breakdown.py --batch 32 --iters 5 --tune-file gpurun_out/cfg/tt_resnet50.json > gpurun_out/cfg/pmc_sq.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/cfg/pmc_fetch -o p -- python3 bench/cnn_breakdown.py --batch 32 --iters 5 --tune-file gpurun_out/cfg/tt_resnet50.json > gpurun_out/cfg/pmc_fetch.log 2>&1 && \
python3 bench/pmc_summary.py gpurun_out/cfg/pmc_sq gpurun_out/cfg/pmc_fetch -o gpurun_out/cfg/pmc_resnet50_forward_r3.json \
  --marker image_to_nhwc --forwards 10 --top 60 --note "ResNet-50 bs32 fp16 forward (eager warmup + graph replay), one counter pass per group" > gpurun_out/cfg/pmc_summary.log 2>&1 && \
echo "pmc ok" >> gpurun_out/cfg/status.txt
