# DCN backward / streaming 1x1 conv / GPU augmentation: parity tests, micro A/Bs, then the bench line (no CPU leg)
set -o pipefail
OUT=gpurun_out/r03g; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_dcn.py tests/test_augment.py tests/test_gpu_conv.py -s > $OUT/tests.log 2>&1; rc=$?; grep -E "^\(|passed|failed|Error" $OUT/tests.log | tail -25; echo tests_rc=$rc
[ $rc -eq 0 ] || exit $rc
for m in 0 1 2; do ADR_DCN_BWD_MODE=$m timeout -k 10 60 python scripts/dcn_bwd_micro.py 2>&1 | grep dcn_bwd || exit 1; done
SPREAD=2.5 timeout -k 10 60 python scripts/dcn_bwd_micro.py 2>&1 | grep dcn_bwd || exit 1
S=40 timeout -k 10 60 python scripts/dcn_bwd_micro.py 2>&1 | grep dcn_bwd || exit 1
S=20 timeout -k 10 60 python scripts/dcn_bwd_micro.py 2>&1 | grep dcn_bwd || exit 1
N=16 C=256 S=160 timeout -k 10 60 python scripts/dcn_bwd_micro.py 2>&1 | grep dcn_bwd || exit 1
ADR_CONV1=1 timeout -k 10 120 python scripts/conv1_ab.py > $OUT/conv1_on.log 2>&1 || { tail $OUT/conv1_on.log; exit 1; }
ADR_CONV1=0 timeout -k 10 120 python scripts/conv1_ab.py > $OUT/conv1_off.log 2>&1 || { tail $OUT/conv1_off.log; exit 1; }
paste -d'\n' $OUT/conv1_on.log $OUT/conv1_off.log | grep conv1
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 --warmup 10 --infer-steps 0 --stage-check 0 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json
python -c "import json;d=json.load(open('$OUT/bench.json'));print('ms_per_step',d['ms_per_step'],'value',d['value'],'events',d['ms_per_step_events'],'augment',d['augment'])"
