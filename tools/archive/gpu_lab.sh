# run a prebuilt GEMM-lab binary (labbin/<name>) on the GPU box: solo + 2-stream timings
set -o pipefail
mkdir -p gpurun_out
for b in "$@"; do
  timeout -k 10 240 ./labbin/$b --iters 50 --concurrent > gpurun_out/lab_$b.txt 2>&1 || exit $?
done
