set -o pipefail
bash tools/gpu_xgmi_cause2.sh
bash tools/gpu_configs_r3.sh
