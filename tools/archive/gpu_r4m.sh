# round 4: fused ResNet stem (image -> space-to-depth -> conv -> ReLU -> max-pool in one kernel):
# numerics, same-box serving A/B vs the three-kernel stem, single-stream forward + kernel table
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r4m
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py -k "stem or s2d or deep" \
  > gpurun_out/r4m/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_models2_gpu.py::test_resnet50_hip_matches_torch \
  tests/test_models_fp32_gpu.py::test_resnet50_hip_vs_fp32 >> gpurun_out/r4m/pytest.log 2>&1 || exit $?
for r in 1 2; do
  i=0
  for arm in "RDB_RESNET_STEM_FUSED=0" "RDB_RESNET_STEM_FUSED=1"; do
    i=$((i+1))
    timeout -k 10 240 env $arm python -u bench/serve_bench.py --model resnet50 --closed 96 --seconds 5 \
      --json-out gpurun_out/r4m/resnet_arm${i}_r$r.json > gpurun_out/r4m/resnet_arm${i}_r$r.log 2>&1 || exit $?
    echo "arm$i [$arm] r$r $(tail -n 1 gpurun_out/r4m/resnet_arm${i}_r$r.log)" >> gpurun_out/r4m/resnet_ab.txt
  done
done
T=ray_dynamic_batching_amd/ops/tuned/mi355x_resnet50_B32_cs2_d4.json
timeout -k 10 200 python -u bench/cnn_breakdown.py --model resnet50 --batch 32 --iters 30 --tune-file $T > gpurun_out/r4m/cnn_breakdown.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4m/profcnn -o c -- \
  python3 bench/cnn_breakdown.py --model resnet50 --batch 32 --iters 20 --tune-file $T > gpurun_out/r4m/prof_cnn.log 2>&1 || exit $?
f=$(ls gpurun_out/r4m/profcnn/*/c_kernel_trace.csv gpurun_out/r4m/profcnn/c_kernel_trace.csv 2>/dev/null | head -n 1)
python3 bench/trace_table.py "$f" --tail 0.5 --marker softmax_topk > gpurun_out/r4m/trace_table_resnet_forward.txt 2>&1
rm -f "$f"
# the 4-wave 256x128 / 128x256 DEEP tiles (128x64 / 64x128 accumulators per wave, spill-free at 1 block / CU)
for shp in "4096 3072 768 --act gelu --bias" "4096 2304 768" "4096 768 3072 --bias --res" "4096 768 768 --bias --res"; do
  set -- $shp
  timeout -k 10 120 python -u bench/gemm_probe.py --m $1 --n $2 --k $3 ${@:4} --iters 100 >> gpurun_out/r4m/gemm_probe.jsonl 2> gpurun_out/r4m/gemm_probe.err || exit $?
done
