# r04e: level-packed AYHead — packed-vs-levels tests, head/GN/DCN/net tests, then the n-scale step A/B
set -o pipefail
OUT=gpurun_out/r04e; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_packed_head.py tests/test_gpu_gn.py tests/test_gpu_dcn.py tests/test_gpu_net.py tests/test_gpu_trainer.py \
  tests/test_gpu_graph.py > $OUT/tests.log 2>&1; rc=$?
tail -30 $OUT/tests.log; echo "tests_rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 40 --warmup 10 --no-cpu-baseline --infer-steps 0 --stage-check 0 --augment-bench 0 \
  > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json
python -c "import json;d=json.load(open('$OUT/bench.json'));print('n', d['ms_per_step'], d['value'], d['host_enqueue_ms_per_step'], d['roofline']['conv_family'])"
exit $rc
