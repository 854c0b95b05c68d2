#!/bin/bash
# Round 6: halo conv patch swizzle chunk ^ (row & 7) (was (row >> 1) & 7): halo GPU tests, bank-conflict
# counters of the ResNet-50 forward, per-layer graph-timed halo variants, single-stream forward and serving.
set -o pipefail
O=gpurun_out/r6ap
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_ops_gpu.py -k "halo" \
    > $O/pytest_halo.log 2>&1 || { tail -30 $O/pytest_halo.log; exit 1; }
tail -n 2 $O/pytest_halo.log
D=ray_dynamic_batching_amd/ops/tuned
B="python3 bench/cnn_breakdown.py --model resnet50 --batch 32 --iters 5 --tune-file $D/mi355x_resnet50_B32_cs1_d2.json"
SQ="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE"
timeout -s KILL 240 rocprofv3 --pmc $SQ --output-format csv -d $O/resnet_sq -o p -- $B > $O/resnet_sq.log 2>&1 || { tail -5 $O/resnet_sq.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $O/resnet_fetch -o p -- $B > $O/resnet_fetch.log 2>&1 || { tail -5 $O/resnet_fetch.log; exit 1; }
python3 bench/pmc_summary.py $O/resnet_sq $O/resnet_fetch -o $O/pmc_resnet_forward_r6_pswz.json --marker softmax_topk --forwards 10 --top 30 \
  --note "ResNet-50 bs32 forward, halo patch swizzle row & 7, single-stream table, graph replay (tools/gpu_r6ap.sh)" > $O/resnet_summary.log 2>&1 || { tail -5 $O/resnet_summary.log; exit 1; }
find $O -name "*.csv" -size +2M -delete
timeout -k 10 300 python bench/conv_halo_bench.py --json-out $O/conv_halo_bench_s1.json > $O/conv_halo_bench_s1.log 2>&1 || { tail -20 $O/conv_halo_bench_s1.log; exit 1; }
timeout -k 10 300 python bench/conv_halo_bench.py --stride 2 --json-out $O/conv_halo_bench_s2.json > $O/conv_halo_bench_s2.log 2>&1 || { tail -20 $O/conv_halo_bench_s2.log; exit 1; }
for i in 1 2; do
  timeout -k 10 200 python -u bench/cnn_breakdown.py --model resnet50 --batch 32 --iters 100 --tune-file $D/mi355x_resnet50_B32_cs1_d2.json > $O/rn_cs1_$i.log 2>&1 || { tail -20 $O/rn_cs1_$i.log; exit 1; }
  echo "resnet cs1 $i $(grep '^{' $O/rn_cs1_$i.log | tail -n 1)"
  timeout -k 10 300 python bench/serve_bench.py --model resnet50 --closed 128 --seconds 5 --json-out $O/rn_c128_$i.json > $O/rn_c128_$i.log 2>&1 || { tail -20 $O/rn_c128_$i.log; exit 1; }
  python3 -c "import json; p=json.load(open('$O/rn_c128_$i.json'))['points'][0]; print('serve c128', p['req_per_s'], p['p50_ms'], p['p99_ms'])"
done
