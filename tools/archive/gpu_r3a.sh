set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_models2_gpu.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3a_models2.log 2>&1; rc=$?
echo "pytest rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3a_bench.log 2>&1
