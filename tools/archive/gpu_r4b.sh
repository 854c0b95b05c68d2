# stream-K GEMM lab: solo + 2-stream timings, correctness of first and last launch
set -o pipefail
mkdir -p gpurun_out/r4b
timeout -k 10 300 ./labbin/sk_lab --iters 50 --concurrent > gpurun_out/r4b/sk_lab.txt 2>&1
