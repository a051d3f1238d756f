# A/B: double-buffered WGRAD tile (ADR_WG_DB=1) vs single buffer; conv / grads tests with it on first
set -o pipefail
OUT=gpurun_out/ab_wgdb; mkdir -p $OUT
ADR_WG_DB=1 timeout -k 10 300 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_conv.py tests/test_gpu_grads.py tests/test_gpu_defer.py > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log; echo "tests_rc=$rc"; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  ADR_WG_DB=$v timeout -k 10 300 python -u bench.py --scale l --img 1280 --bs 16 --steps 10 --warmup 3 --roofline-steps 0 \
    --stage-check 0 --no-cpu-baseline --infer-steps 0 --augment-bench 0 > $OUT/l_$v.log 2>&1 || { tail -20 $OUT/l_$v.log; exit 1; }
  python -c "import json;a=[json.loads(l) for l in open('$OUT/l_$v.log') if l.startswith('{')][-1];print('l $v',a['ms_per_step'])"
done
for v in 0 1 0 1; do
  ADR_WG_DB=$v timeout -k 10 300 python -u bench.py --steps 40 --warmup 10 --no-cpu-baseline --infer-steps 0 --stage-check 0 \
    --augment-bench 0 --roofline-steps 0 > $OUT/n_$v.log 2>&1 || { tail -20 $OUT/n_$v.log; exit 1; }
  python -c "import json;a=[json.loads(l) for l in open('$OUT/n_$v.log') if l.startswith('{')][-1];print('n $v',a['ms_per_step'])"
done
