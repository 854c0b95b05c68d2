# round 4: ResNet-50 kernels (avgpool rewrite, space-to-depth stem, split-K convolutions,
# 1x1 convs on the dense GEMM tiles) -- numerics, a same-box serving A/B, single-stream
# forward times, kernel traces of the forward and of the serving run
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r4g
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py \
  -k "avgpool or s2d or conv2d or pools or image_to or softmax_topk" tests/test_models2_gpu.py::test_resnet50_hip_matches_torch \
  tests/test_models_fp32_gpu.py::test_resnet50_hip_vs_fp32 > gpurun_out/r4g/pytest_resnet.log 2>&1 || exit $?
for r in 1 2; do
  i=0
  for arm in "RDB_CONV1X1_GEMM=0 RDB_CONV_SPLITK=0 RDB_RESNET_S2D=0" "RDB_TUNE_FILE=gpurun_out/r4g/tiles_new_r$r.json" \
             "RDB_CONV_SPLITK=0 RDB_TUNE_FILE=gpurun_out/r4g/tiles_nosk_r$r.json" \
             "RDB_TUNE_STREAMS=2 RDB_TUNE_FILE=gpurun_out/r4g/tiles_ts2_r$r.json"; do
    i=$((i+1))
    timeout -k 10 240 env $arm python -u bench/serve_bench.py --model resnet50 --closed 96 --seconds 5 \
      --json-out gpurun_out/r4g/resnet_arm${i}_r$r.json > gpurun_out/r4g/resnet_arm${i}_r$r.log 2>&1 || exit $?
    echo "arm$i [$arm] r$r $(tail -n 1 gpurun_out/r4g/resnet_arm${i}_r$r.log)" >> gpurun_out/r4g/resnet_ab.txt
  done
done
T=gpurun_out/r4g/tiles_new_r1.json
timeout -k 10 200 python -u bench/cnn_breakdown.py --model resnet50 --batch 32 --iters 30 --tune-file $T > gpurun_out/r4g/cnn_breakdown_new.log 2>&1 || exit $?
timeout -k 10 200 env RDB_CONV1X1_GEMM=0 RDB_CONV_SPLITK=0 RDB_RESNET_S2D=0 python -u bench/cnn_breakdown.py --model resnet50 --batch 32 --iters 30 \
  --tune-file ray_dynamic_batching_amd/ops/tuned/mi355x_resnet50_B32_d2.json > gpurun_out/r4g/cnn_breakdown_old.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4g/profcnn -o c -- \
  python3 bench/cnn_breakdown.py --model resnet50 --batch 32 --iters 20 --tune-file $T > gpurun_out/r4g/prof_cnn.log 2>&1 || exit $?
f=$(ls gpurun_out/r4g/profcnn/*/c_kernel_trace.csv gpurun_out/r4g/profcnn/c_kernel_trace.csv 2>/dev/null | head -n 1)
python3 bench/trace_table.py "$f" --tail 0.5 --marker softmax_topk > gpurun_out/r4g/trace_table_resnet_forward.txt 2>&1
rm -f "$f"
RDB_TUNE_FILE=$T timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4g/prof -o s -- \
  python3 bench/serve_bench.py --model resnet50 --closed 96 --seconds 4 > gpurun_out/r4g/prof_serve.log 2>&1 || exit $?
f=$(ls gpurun_out/r4g/prof/*/s_kernel_trace.csv gpurun_out/r4g/prof/s_kernel_trace.csv 2>/dev/null | head -n 1)
python3 bench/trace_gaps.py "$f" --tail 0.3 > gpurun_out/r4g/trace_gaps_resnet_serving.txt 2>&1
python3 bench/trace_table.py "$f" --tail 0.3 --marker softmax_topk > gpurun_out/r4g/trace_table_resnet_serving.txt 2>&1
rm -f "$f"
