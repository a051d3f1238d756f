# r04k: configs[4] (l-scale 1280^2 bs 16) after the packed head: tests, bf16 bench, fp8 bench, replay profile
set -o pipefail
OUT=gpurun_out/r04k; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 500 --timeout-method thread -m gpu tests/test_gpu_dcn.py tests/test_gpu_lscale.py \
  > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; echo "tests_rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --scale l --img 1280 --bs 16 --steps 10 --warmup 3 --roofline-steps 0 --stage-check 0 \
  --no-cpu-baseline --infer-steps 0 --augment-bench 0 > $OUT/l.log 2>&1 || { tail -20 $OUT/l.log; exit 1; }
grep '^{' $OUT/l.log | tail -1 > $OUT/l.json
timeout -k 10 400 python -u bench.py --scale l --img 1280 --bs 16 --steps 10 --warmup 3 --roofline-steps 0 --stage-check 0 \
  --no-cpu-baseline --infer-steps 0 --augment-bench 0 --conv-fp8 > $OUT/l_fp8.log 2>&1 || { tail -20 $OUT/l_fp8.log; exit 1; }
grep '^{' $OUT/l_fp8.log | tail -1 > $OUT/l_fp8.json
python -c "import json;a=json.load(open('$OUT/l.json'));b=json.load(open('$OUT/l_fp8.json'));print('l bf16',a['ms_per_step'],a['value'],'fp8',b['ms_per_step'],b['value'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python3 bench.py --scale l --img 1280 --bs 16 --steps 4 --warmup 2 --roofline-steps 0 --stage-check 0 --no-cpu-baseline --infer-steps 0 --augment-bench 0 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python scripts/replay_breakdown.py $OUT/prof/run_kernel_trace.csv --steps 3 --top 40 > $OUT/replay.md && head -16 $OUT/replay.md
gzip -f $OUT/prof/run_kernel_trace.csv
