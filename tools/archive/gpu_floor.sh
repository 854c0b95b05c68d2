# Kernel fixed-cost probe under several HIP runtime settings (bench/launch_floor.py).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/launch_floor.jsonl
: > $out
for e in "X=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "HIP_FORCE_DEV_KERNARG=1" "ROC_SYSTEM_SCOPE_SIGNAL=0" "AMD_DIRECT_DISPATCH=0" "ROC_ACTIVE_WAIT_TIMEOUT=100"; do
  timeout -k 10 120 env $e python -u bench/launch_floor.py >> $out 2> gpurun_out/launch_floor.err || exit 1
done
grep -v amdgpu.ids $out
