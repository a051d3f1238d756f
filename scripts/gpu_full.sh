# Round evidence in one GPU call: the -m gpu suite, the default bench line (bench.py with no flags), a rocprofv3
# kernel-trace summary of a short bench run and the two PMC passes of the traffic table.
# usage: bash scripts/gpu_full.sh <tag>
set -o pipefail
TAG=${1:-full}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu tests \
  > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; echo "tests_rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 500 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json
python -c "import json;d=json.load(open('$OUT/bench.json'));print('ms_per_step',d['ms_per_step'],'value',d['value'],'events',d['ms_per_step_events'],'staging',d['ddp_staging'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --infer-steps 0 --roofline-steps 0 --stage-check 0 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
bash scripts/pmc_bench_traffic.sh && cp gpurun_out/pmc_bench/pmc_traffic.json $OUT/pmc_traffic.json
exit $rc
