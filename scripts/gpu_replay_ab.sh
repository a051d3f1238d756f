# Same-box kernel-trace A/B of two environment settings over the replayed bench steps:
# bash scripts/gpu_replay_ab.sh <tag> "<envA>" "<envB>"  -> gpurun_out/<tag>/{A,B}_replay.md (replay_breakdown tables)
set -o pipefail
TAG=$1; A=$2; B=$3; OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in A B; do
  E=$([ $v = A ] && echo "$A" || echo "$B")
  export $E
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/$v -o run -- python bench.py --steps 10 --warmup 2 --roofline-steps 0 --infer-steps 0 --no-cpu-baseline --stage-check 0 --augment-bench 0 > $OUT/$v.log 2>&1 || { echo ${v}_failed; tail -20 $OUT/$v.log; exit 1; }
  unset ${E%%=*}
  python scripts/replay_breakdown.py $(find $OUT/$v -name "*kernel_trace.csv" | head -1) --top 80 > $OUT/${v}_replay.md
  rm -rf $OUT/$v
  echo "$v [$E]: $(head -1 $OUT/${v}_replay.md)"
done
