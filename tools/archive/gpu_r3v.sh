# same-box A/B of the residual prefetch: GEMM probes, then the headline bench (3 rounds)
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r3v
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=ray_dynamic_batching_amd/_variants/noprefetch/_rdb_ops.cpython-310-x86_64-linux-gnu.so
P="timeout -k 10 120 python -u bench/gemm_probe.py --iters 400 --bias --res"
for arm in A B; do
  if [ $arm = A ]; then export RDB_OPS_SO=$V; else unset RDB_OPS_SO; fi
  $P --m 4096 --n 768 --k 3072 --cfg 19 > gpurun_out/r3v/d_$arm.log 2>&1 || exit $?
  $P --m 4096 --n 768 --k 768 --cfg 10 > gpurun_out/r3v/o_$arm.log 2>&1 || exit $?
done
unset RDB_OPS_SO
for f in gpurun_out/r3v/*_[AB].log; do echo "$f $(grep -o '"ours[^}]*}' $f)" >> gpurun_out/r3v/probe_summary.txt; done
bash tools/gpu_ab_env.sh 3 "RDB_OPS_SO=$V" "RDB_AB_PREFETCH=1"
