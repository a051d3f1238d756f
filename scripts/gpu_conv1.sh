set -o pipefail
OUT=gpurun_out/conv1; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_net.py tests/test_gpu_predictor.py tests/test_gpu_yolo11.py > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; echo tests_rc=$rc
[ $rc -eq 0 ] || exit $rc
ADR_CONV1=1 timeout -k 10 120 python scripts/conv1_ab.py > $OUT/conv1_on.log 2>&1 || { tail $OUT/conv1_on.log; exit 1; }
ADR_CONV1=0 timeout -k 10 120 python scripts/conv1_ab.py > $OUT/conv1_off.log 2>&1 || { tail $OUT/conv1_off.log; exit 1; }
paste -d'\n' $OUT/conv1_on.log $OUT/conv1_off.log | grep conv1 | tail -16
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 --warmup 10 --infer-steps 10 --stage-check 0 --augment-bench 0 --roofline-steps 0 > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 1; }
python -c "import json;d=[json.loads(l) for l in open('$OUT/b.log') if l.startswith('{')][-1];print('n', d['ms_per_step'], d['ms_per_step_events']['median'], 'infer', d['inference']['value'])"
timeout -k 10 600 python -u bench.py --scale l --img 1280 --bs 16 --steps 10 --warmup 3 --roofline-steps 0 --stage-check 0 > $OUT/l.log 2>&1 || { tail -20 $OUT/l.log; exit 1; }
python -c "import json;d=[json.loads(l) for l in open('$OUT/l.log') if l.startswith('{')][-1];print('l', d['ms_per_step'], d['value'])"
