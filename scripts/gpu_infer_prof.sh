# Kernel-trace profile of the batched-inference bench (BASELINE.json configs[1]) only.
# usage: bash scripts/gpu_infer_prof.sh <tag>   (outputs under gpurun_out/<tag>/)
set -o pipefail
TAG=${1:-inf}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python bench.py --infer --infer-steps 20 > $OUT/infer.log 2>&1 || { tail -20 $OUT/infer.log; exit 1; }
grep '^{' $OUT/infer.log | tail -1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --infer --infer-steps 50 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv"
