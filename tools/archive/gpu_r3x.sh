# FFN-down tile A/B in the two-stream bench: shipped (cfg 19) vs pp 256x144 (20), pp 128x256 (21), 8-wave 256x128 (13)
T=$GRAFT_REPO_ROOT/tools/ab_tables_r3s
bash tools/gpu_ab_env.sh 3 "RDB_AB_SHIPPED=1" "RDB_TUNE_FILE=$T/ffn2_cfg20.json" "RDB_TUNE_FILE=$T/ffn2_cfg21.json" "RDB_TUNE_FILE=$T/ffn2_cfg13.json"
