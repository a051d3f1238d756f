# a -k subset of the GPU tests, then two short bench lines (no CPU leg, no inference, no staging, no augmentation)
set -o pipefail
OUT=gpurun_out/quick; mkdir -p $OUT
K="${1:-conv}"
timeout -k 10 300 python -u -m pytest -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu -k "$K" tests > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; echo tests_rc=$rc
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 --warmup 10 --infer-steps 0 --stage-check 0 --augment-bench 0 --roofline-steps 0 > $OUT/b$i.log 2>&1 || { tail $OUT/b$i.log; exit 1; }
python -c "import json;d=[json.loads(l) for l in open('$OUT/b$i.log') if l.startswith('{')][-1];print('bench', d['ms_per_step'], d['ms_per_step_events']['median'])"; done
