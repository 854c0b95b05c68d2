# round 4: DEEP tiles + pstats numerics; BERT GEMM shapes standalone (all tiles, DEEP, stream-K)
# vs hipBLASLt; same-box BERT A/B (LayerNorm folded with partial statistics) and ResNet A/B (DEEP)
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r4l
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ln_staged_gpu.py \
  tests/test_ops_gpu.py -k "ln_staged or partial or pstats or deep or splitk or conv2d" > gpurun_out/r4l/pytest.log 2>&1 || exit $?
for shp in "4096 3072 768 --act gelu --bias" "4096 768 3072 --bias --res --streamk 192" "4096 2304 768" "4096 768 768 --bias --res --streamk 192"; do
  set -- $shp
  timeout -k 10 120 python -u bench/gemm_probe.py --m $1 --n $2 --k $3 ${@:4} --iters 100 >> gpurun_out/r4l/gemm_probe.jsonl 2> gpurun_out/r4l/gemm_probe.err || exit $?
done
rm -f gpurun_out/abe/summary.txt
bash tools/gpu_ab_env.sh 2 "RDB_AB=0" "RDB_BERT_LN_PSTATS=1" || exit $?
cp gpurun_out/abe/summary.txt gpurun_out/r4l/bert_ab.txt
for r in 1 2; do
  i=0
  for arm in "RDB_GEMM_DEEP=0 RDB_TUNE_STREAMS=2 RDB_TUNE_FILE=gpurun_out/r4l/tiles_nodeep_r$r.json" \
             "RDB_TUNE_STREAMS=2 RDB_TUNE_FILE=gpurun_out/r4l/tiles_deep_r$r.json"; do
    i=$((i+1))
    timeout -k 10 240 env $arm python -u bench/serve_bench.py --model resnet50 --closed 96 --seconds 5 \
      --json-out gpurun_out/r4l/resnet_arm${i}_r$r.json > gpurun_out/r4l/resnet_arm${i}_r$r.log 2>&1 || exit $?
    echo "arm$i [$arm] r$r $(tail -n 1 gpurun_out/r4l/resnet_arm${i}_r$r.log)" >> gpurun_out/r4l/resnet_ab.txt
  done
done
T=gpurun_out/r4l/tiles_deep_r1.json
timeout -k 10 200 python -u bench/cnn_breakdown.py --model resnet50 --batch 32 --iters 30 --tune-file $T > gpurun_out/r4l/cnn_breakdown.log 2>&1
