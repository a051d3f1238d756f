# GPU parity tests (+ optional bench line). usage: bash scripts/gpu_tests.sh <tag> [pytest args...]
# Each GPU step has its own time limit; steps are chained so a failure ends the call.
set -o pipefail
TAG=${1:-tests}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu "$@" \
  > $OUT/gpu_tests.log 2>&1
rc=$?
echo "tests_rc=$rc"; grep -E "passed|failed|error" $OUT/gpu_tests.log | tail -5
exit $rc
