# iteration loop on the GPU box: all gpu tests, bench line, rocprof kernel stats, conv table.
# usage: bash scripts/gpu_iter.sh <tag>
set -o pipefail
TAG=${1:-iter}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -15 $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --no-cpu-baseline > $OUT/bench.log 2>&1 || { echo bench_failed; tail -30 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json; cut -c1-400 $OUT/bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/prof.log 2>&1 || { echo prof_failed; tail -20 $OUT/prof.log; exit 1; }
echo prof_ok
timeout -k 10 300 python scripts/conv_table.py > $OUT/conv_table.txt 2>&1 || { echo table_failed; tail -5 $OUT/conv_table.txt; exit 1; }
echo table_ok
