set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_ffn2_12 -o p -- python3 bench/gemm_probe.py --m 4096 --n 768 --k 3072 --bias --res --cfg 12 --iters 20 && \
timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_ffn2_9 -o p -- python3 bench/gemm_probe.py --m 4096 --n 768 --k 3072 --bias --res --cfg 9 --iters 20 && \
timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_ffn1_4 -o p -- python3 bench/gemm_probe.py --m 4096 --n 3072 --k 768 --bias --act gelu --cfg 4 --iters 20 && \
timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_qkv_8 -o p -- python3 bench/gemm_probe.py --m 4096 --n 2304 --k 768 --bias --cfg 8 --iters 20
