# NMS tests, then kernel-trace medians with the distributed max_nms select (default) and without (ADR_NMS_DSEL=0)
set -o pipefail
mkdir -p gpurun_out/dsel
timeout -k 10 300 python -u -m pytest tests/test_gpu_nms.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dsel/tests.log 2>&1 || { tail -30 gpurun_out/dsel/tests.log; exit 1; }
tail -1 gpurun_out/dsel/tests.log
bash scripts/gpu_nms_trace.sh dsel_on "0" && ADR_NMS_DSEL=0 bash scripts/gpu_nms_trace.sh dsel_off "0"
