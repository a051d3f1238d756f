# One build -> measure iteration on the GPU box: the whole -m gpu suite (or a -k subset), the bench line (no CPU
# leg) and a rocprofv3 kernel-trace summary of a short bench run. Each step has its own time limit and the chain
# stops at the first failure.   usage: bash scripts/gpu_cycle.sh <tag> ["<pytest -k expr>"] [bench args...]
set -o pipefail
TAG=${1:-cyc}; K=${2:-}; shift 2 2>/dev/null || shift $#
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 400 python -u -m pytest -q -p no:cacheprovider --timeout 120 --timeout-method thread --maxfail 8 \
  -m gpu "${KA[@]}" tests > $OUT/tests.log 2>&1
rc=$?; tail -15 $OUT/tests.log; echo "tests_rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 --infer-steps 0 "$@" > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json
python -c "import json;d=json.load(open('$OUT/bench.json'));print('ms_per_step',d['ms_per_step'],'value',d['value'],'host_ms',d.get('host_enqueue_ms_per_step'))"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --infer-steps 0 --roofline-steps 0 "$@" > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
exit $rc
