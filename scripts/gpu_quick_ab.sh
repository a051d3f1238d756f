# quick iteration: named GPU tests, then the n-scale bench line (no CPU leg / inference / staging legs) and a replay profile
# usage: bash scripts/gpu_quick_ab.sh <tag> "<pytest targets>"
set -o pipefail
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu $2 \
    > $OUT/tests.log 2>&1; rc=$?
  tail -15 $OUT/tests.log; echo "tests_rc=$rc"
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py --steps 40 --warmup 10 --no-cpu-baseline --infer-steps 0 --stage-check 0 --augment-bench 0 \
  > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json
python -c "import json;d=json.load(open('$OUT/bench.json'));print('n', d['ms_per_step'], d['value'], d['host_enqueue_ms_per_step'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --infer-steps 0 --roofline-steps 0 --stage-check 0 --augment-bench 0 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python scripts/replay_breakdown.py $OUT/prof/run_kernel_trace.csv --top 30 > $OUT/replay.md && head -16 $OUT/replay.md
rm -f $OUT/prof/run_kernel_trace.csv.gz; gzip -f $OUT/prof/run_kernel_trace.csv
