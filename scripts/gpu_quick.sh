# quick GPU loop: selected tests + the bench line (no profile). usage: bash scripts/gpu_quick.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-quick}; K=${2:-}
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ -n "$K" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -k "$K" > $OUT/gpu_tests.log 2>&1
else
  timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > $OUT/gpu_tests.log 2>&1
fi
echo "tests_rc=$?"; tail -6 $OUT/gpu_tests.log
timeout -k 10 600 python bench.py --no-cpu-baseline > $OUT/bench.log 2>&1 || { echo bench_failed; tail -30 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json; cat $OUT/bench.json
