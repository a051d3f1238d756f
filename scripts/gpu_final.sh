# Round evidence in one GPU call: the -m gpu suite, the default bench line (bench.py with no flags), a rocprofv3
# kernel-trace (stats + replayed-step breakdown) of a short bench run, the two PMC traffic passes, the l-scale line.
# usage: bash scripts/gpu_final.sh <tag>
set -o pipefail
TAG=${1:-final}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests \
  > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; echo "tests_rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 500 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json
python -c "import json;d=json.load(open('$OUT/bench.json'));print('ms_per_step',d['ms_per_step'],'value',d['value'],'events',d['ms_per_step_events'],'host',d['host_enqueue_ms_per_step'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --infer-steps 0 --roofline-steps 0 --stage-check 0 --augment-bench 0 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
cp $OUT/prof/run_kernel_stats.csv $OUT/kernel_stats.csv
python scripts/replay_breakdown.py $OUT/prof/run_kernel_trace.csv --top 40 > $OUT/replay.md && head -16 $OUT/replay.md
gzip -f $OUT/prof/run_kernel_trace.csv
bash scripts/pmc_bench_traffic.sh && cp gpurun_out/pmc_bench/pmc_traffic.json $OUT/pmc_traffic.json || exit 1
timeout -k 10 400 python -u bench.py --scale l --img 1280 --bs 16 --steps 10 --warmup 3 --roofline-steps 0 --stage-check 0 \
  --no-cpu-baseline --infer-steps 0 --augment-bench 0 > $OUT/l.log 2>&1 || { tail -20 $OUT/l.log; exit 1; }
grep '^{' $OUT/l.log | tail -1 > $OUT/l.json
python -c "import json;a=json.load(open('$OUT/l.json'));print('l bf16',a['ms_per_step'],a['value'])"
exit $rc
