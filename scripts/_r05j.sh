set -o pipefail
timeout -k 10 300 python scripts/conv_table.py --by-gap > gpurun_out/r05j_conv.txt 2>&1 || exit 1
bash scripts/ab_env2.sh r05j1 "ADR_BN_BSTAT=1" "ADR_BN_BSTAT=0" 2 > gpurun_out/r05j.txt 2>&1 || exit 1
bash scripts/ab_env2.sh r05j2 "ADR_BN_XF_FWD=1" "ADR_BN_XF_FWD=0" 2 >> gpurun_out/r05j.txt 2>&1
