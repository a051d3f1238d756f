# r04j: whole -m gpu suite, then the n-scale bench A/B pair (fused gate backward on / via the reduce + x kernels) and a replay profile
set -o pipefail
OUT=gpurun_out/r04j; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests \
  > $OUT/tests.log 2>&1; rc=$?
tail -12 $OUT/tests.log; echo "tests_rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/gpu_quick_ab.sh r04j_b "" || exit 1
exit $rc
