# stream-K lab, then the round-4 first-look bench / trace
set -o pipefail
bash tools/gpu_r4b.sh || exit $?
bash tools/gpu_r4a.sh
