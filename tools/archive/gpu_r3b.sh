set -o pipefail
bash tools/fresh.sh || exit 9
bash tools/gpu_xgmi_cause.sh
bash tools/gpu_tp8c.sh
