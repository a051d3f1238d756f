# One iteration of the build -> measure loop: a pytest subset (-k expression), the bench line, and a rocprofv3
# kernel-trace summary of a short bench run. usage: bash scripts/gpu_check.sh <tag> "<pytest -k expr>"
set -o pipefail
TAG=${1:-chk}; OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu -k "$2" tests \
    > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
  tail -2 $OUT/tests.log
fi
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --infer-steps 0 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $OUT/bench.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --infer-steps 0 --roofline-steps 0 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv"
