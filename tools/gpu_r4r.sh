# round 4: per-batch model profiles (fork CSV contract, graph mode) of the CNN zoo on the round-4
# kernels (split-K / dense-tile conv candidates, fused ResNet stem), vs the reference's A6000 CSVs
set -o pipefail
bash tools/fresh.sh || exit 9
mkdir -p gpurun_out/r4r
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u bench/profile_models.py --models resnet50,shufflenet-v2,efficientnet-v2s --batches 1,32,256 \
  --out gpurun_out/r4r/model_profiles > gpurun_out/r4r/profile_models.log 2>&1
