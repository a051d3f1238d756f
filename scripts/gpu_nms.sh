# adr_nms micro timing + per-kernel split. usage: bash scripts/gpu_nms.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-nms}; OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ -n "$2" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_nms.py -x -q --timeout 120 --timeout-method thread -k "$2" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
  tail -2 $OUT/tests.log
fi
for m in ${MODES:-default}; do
  ADR_NMS_MODE=${m%%:*} ADR_NMS_BAR=${m##*:} timeout -k 10 200 python scripts/nms_micro.py 50 > $OUT/micro_$m.log 2>&1 || { tail -20 $OUT/micro_$m.log; exit 1; }
  tail -1 $OUT/micro_$m.log
done
for st in ${STOPS}; do
  ADR_NMS_BAR=${BAR:-1} ADR_NMS_STOP=$st timeout -k 10 200 python scripts/nms_micro.py 30 > $OUT/stop_$st.log 2>&1 || { tail -20 $OUT/stop_$st.log; exit 1; }
  tail -1 $OUT/stop_$st.log
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 scripts/nms_micro.py 50 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); grep -i nms $f | cut -c1-150
