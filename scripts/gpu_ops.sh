# GPU iteration: all gpu tests, bench line (no CPU leg), per-entry-point op table.
# usage: bash scripts/gpu_ops.sh <tag>
set -o pipefail
TAG=${1:-ops}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -8 $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.log 2>&1 || { echo bench_failed; tail -30 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json; cut -c1-300 $OUT/bench.json
timeout -k 10 300 python scripts/op_table.py > $OUT/op_table.txt 2>&1 || { echo optable_failed; tail -20 $OUT/op_table.txt; exit 1; }
echo optable_ok
