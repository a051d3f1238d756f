# r04d: the vectorised split-K reduce — conv / deferral / gradient tests, then the n-scale and l-scale step
set -o pipefail
OUT=gpurun_out/r04d; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_conv.py tests/test_gpu_defer.py tests/test_gpu_grads.py tests/test_gpu_dcn.py tests/test_gpu_trainer.py \
  tests/test_gpu_bf16_train.py tests/test_gpu_stages.py > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log; echo "tests_rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 40 --warmup 10 --no-cpu-baseline --infer-steps 0 --stage-check 0 --augment-bench 0 \
  > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json
python -c "import json;d=json.load(open('$OUT/bench.json'));print('n', d['ms_per_step'], d['value'], d['host_enqueue_ms_per_step'], d['roofline']['conv_family'])"
timeout -k 10 400 python -u bench.py --scale l --img 1280 --bs 16 --steps 10 --warmup 3 --roofline-steps 0 --stage-check 0 \
  > $OUT/l.log 2>&1 || { tail -20 $OUT/l.log; exit 1; }
grep '^{' $OUT/l.log | tail -1 > $OUT/l.json
python -c "import json;d=json.load(open('$OUT/l.json'));print('l', d['ms_per_step'], d['value'])"
exit $rc
