# round 4: ResNet-50 after the fast im2col path / packed head / header zeroing: numerics,
# serving A/B (1 vs 2 compute streams), single-stream forward + per-kernel table, Poisson curve
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r4j
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py \
  -k "avgpool or s2d or conv2d or pools or image_to or softmax_topk" tests/test_models2_gpu.py::test_resnet50_hip_matches_torch \
  tests/test_models_fp32_gpu.py::test_resnet50_hip_vs_fp32 > gpurun_out/r4j/pytest_resnet.log 2>&1 || exit $?
for r in 1 2; do
  i=0
  for arm in "RDB_TUNE_FILE=gpurun_out/r4j/tiles_cs1_r$r.json -- --compute-streams 1 --pipeline-depth 2" \
             "RDB_TUNE_FILE=gpurun_out/r4j/tiles_cs2_r$r.json -- --compute-streams 2 --pipeline-depth 4" \
             "RDB_TUNE_STREAMS=2 RDB_TUNE_FILE=gpurun_out/r4j/tiles_cs2t2_r$r.json -- --compute-streams 2 --pipeline-depth 4"; do
    i=$((i+1))
    envs="${arm%%--*}"; flags="${arm#*-- }"
    timeout -k 10 240 env $envs python -u bench/serve_bench.py --model resnet50 --closed 96 --seconds 5 $flags \
      --json-out gpurun_out/r4j/resnet_arm${i}_r$r.json > gpurun_out/r4j/resnet_arm${i}_r$r.log 2>&1 || exit $?
    echo "arm$i [$arm] r$r $(tail -n 1 gpurun_out/r4j/resnet_arm${i}_r$r.log)" >> gpurun_out/r4j/resnet_ab.txt
  done
done
T=gpurun_out/r4j/tiles_cs1_r1.json
timeout -k 10 200 python -u bench/cnn_breakdown.py --model resnet50 --batch 32 --iters 30 --tune-file $T > gpurun_out/r4j/cnn_breakdown.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4j/profcnn -o c -- \
  python3 bench/cnn_breakdown.py --model resnet50 --batch 32 --iters 20 --tune-file $T > gpurun_out/r4j/prof_cnn.log 2>&1 || exit $?
f=$(ls gpurun_out/r4j/profcnn/*/c_kernel_trace.csv gpurun_out/r4j/profcnn/c_kernel_trace.csv 2>/dev/null | head -n 1)
python3 bench/trace_table.py "$f" --tail 0.5 --marker softmax_topk > gpurun_out/r4j/trace_table_resnet_forward.txt 2>&1
rm -f "$f"
