# r04a: the tests touched this round, then the default bench line (no CPU baseline)
set -o pipefail
OUT=gpurun_out/r04a; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_conv.py::test_conv3_wide_tile_bf16 tests/test_gpu_bnxf.py tests/test_metrics.py tests/test_gpu_nms.py tests/test_gpu_rccl.py tests/test_gpu_bf16_train.py \
  tests/test_gpu_dcn.py tests/test_gpu_predictor.py tests/test_gpu_lscale.py > $OUT/tests.log 2>&1; rc=$?
tail -5 $OUT/tests.log; echo "tests_rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python bench.py --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json
python -c "import json;d=json.load(open('$OUT/bench.json'));print('ms_per_step',d['ms_per_step'],'value',d['value'],'staging',d['ddp_staging'],'nms',d['nms'],'infer',d['inference'])"
exit $rc
