# Kernel-trace medians of adr_nms per nms_micro setting for each ADR_NMS_STOP value (and the chain).
# usage: bash scripts/gpu_nms_trace.sh <tag> "<stops>"
set -o pipefail
TAG=${1:-nmst}; OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for st in ${2:-0}; do
  if [ "$st" = chain ]; then export ADR_NMS_MODE=chain; unset ADR_NMS_STOP; else unset ADR_NMS_MODE; export ADR_NMS_STOP=$st; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/p_$st -o run -- python3 scripts/nms_micro.py 50 > $OUT/p_$st.log 2>&1 || { tail -20 $OUT/p_$st.log; exit 1; }
  f=$(find $OUT/p_$st -name "*kernel_trace.csv" | head -1)
  echo "stop=$st $(python scripts/nms_trace.py $f)"
done
