set -o pipefail
OUT=gpurun_out/dcn1; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_dcn.py tests/test_augment.py -s > $OUT/tests.log 2>&1; rc=$?; grep -E "^\(|passed|failed|Error" $OUT/tests.log | tail -25; echo tests_rc=$rc
[ $rc -eq 0 ] || exit $rc
for m in 0 1 2; do ADR_DCN_BWD_MODE=$m timeout -k 10 60 python scripts/dcn_bwd_micro.py 2>&1 | grep dcn_bwd || exit 1; done
SPREAD=2.5 timeout -k 10 60 python scripts/dcn_bwd_micro.py 2>&1 | grep dcn_bwd || exit 1
S=40 timeout -k 10 60 python scripts/dcn_bwd_micro.py 2>&1 | grep dcn_bwd || exit 1
S=20 timeout -k 10 60 python scripts/dcn_bwd_micro.py 2>&1 | grep dcn_bwd || exit 1
N=16 C=256 S=160 timeout -k 10 60 python scripts/dcn_bwd_micro.py 2>&1 | grep dcn_bwd || exit 1
