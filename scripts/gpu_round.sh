# One GPU session: parity tests, the bench line, and a kernel-trace profile of the bench.
# usage: bash scripts/gpu_round.sh <tag>   (outputs under gpurun_out/<tag>/)
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > $OUT/gpu_tests.log 2>&1
echo "tests_rc=$?"; tail -8 $OUT/gpu_tests.log
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || { echo bench_failed; tail -20 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json; cat $OUT/bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/prof.log 2>&1 || { echo prof_failed; tail -20 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*stats*"
