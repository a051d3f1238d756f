set -o pipefail
bash scripts/ab_env2.sh r05k1 "ADR_BN_XF_MAX_REUSE=150" "ADR_BN_XF_MAX_REUSE=300" 2 > gpurun_out/r05k.txt 2>&1 || exit 1
bash scripts/ab_env2.sh r05k2 "ADR_BN_XF_MAX_REUSE=150" "ADR_BN_XF_MAX_REUSE=100" 1 >> gpurun_out/r05k.txt 2>&1 || exit 1
bash scripts/ab_env2.sh r05k3 "ADR_BN_XF_FWD_MAX_REUSE=200" "ADR_BN_XF_FWD_MAX_REUSE=400" 2 >> gpurun_out/r05k.txt 2>&1 || exit 1
