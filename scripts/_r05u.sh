set -o pipefail
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu -k "wgrad_bias or conv or bf16 or grads or trainer or packed or graph or abi" tests > gpurun_out/r05u_tests.log 2>&1; rc=$?; tail -4 gpurun_out/r05u_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_env3.sh r05v_fb 2 "ADR_FUSE_WG_BIAS=0" "ADR_FUSE_WG_BIAS=1"
