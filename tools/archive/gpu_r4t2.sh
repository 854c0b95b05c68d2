# round 4 final tree: ResNet-50 serving (shipped table) x2 -- regression check after the SwiGLU epilogue change
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r4t2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 1 2; do
  timeout -k 10 240 python -u bench/serve_bench.py --model resnet50 --closed 96 --seconds 5 \
    > gpurun_out/r4t2/resnet_r$r.log 2>&1 || exit $?
done
