# residual-epilogue cost: the BERT o-proj / FFN-down GEMMs with and without the residual operand
set -o pipefail
mkdir -p gpurun_out/r3t
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export RDB_NO_AUTOBUILD=1
P="timeout -k 10 120 python -u bench/gemm_probe.py --iters 400 --bias"
$P --m 4096 --n 768 --k 768 --cfg 10 > gpurun_out/r3t/o_nores.log 2>&1 && \
$P --m 4096 --n 768 --k 768 --cfg 10 --res > gpurun_out/r3t/o_res.log 2>&1 && \
$P --m 4096 --n 768 --k 3072 --cfg 19 > gpurun_out/r3t/d_nores.log 2>&1 && \
$P --m 4096 --n 768 --k 3072 --cfg 19 --res > gpurun_out/r3t/d_res.log 2>&1
rc=$?
for f in gpurun_out/r3t/*.log; do echo "$f $(grep -o '"ours[^}]*}' $f)"; done
exit $rc
