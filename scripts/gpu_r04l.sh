# r04l: whole -m gpu suite, n-scale bench + replay profile, l-scale bench
set -o pipefail
OUT=gpurun_out/r04l; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests \
  > $OUT/tests.log 2>&1; rc=$?
tail -12 $OUT/tests.log; echo "tests_rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/gpu_quick_ab.sh r04l_b "" || exit 1
timeout -k 10 400 python -u bench.py --scale l --img 1280 --bs 16 --steps 10 --warmup 3 --roofline-steps 0 --stage-check 0 \
  --no-cpu-baseline --infer-steps 0 --augment-bench 0 > $OUT/l.log 2>&1 || { tail -20 $OUT/l.log; exit 1; }
grep '^{' $OUT/l.log | tail -1 > $OUT/l.json
python -c "import json;a=json.load(open('$OUT/l.json'));print('l bf16',a['ms_per_step'],a['value'])"
exit $rc
