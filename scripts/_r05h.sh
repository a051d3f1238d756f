set -o pipefail
bash scripts/ab_env2.sh r05h3 "ADR_XF_CONV3=1" "ADR_XF_CONV3=0" 2 > gpurun_out/r05h.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bnxf.py tests/test_gpu_bstat.py tests/test_gpu_dg2.py >> gpurun_out/r05h.txt 2>&1
