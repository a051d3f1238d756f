# Profile pass for the committed evidence: default bench line (with the CPU leg), rocprofv3 kernel stats of the
# same command, and two PMC passes (FETCH_SIZE, WRITE_SIZE) for HBM traffic per launch.
# usage: bash scripts/gpu_prof.sh <tag>
set -o pipefail
TAG=${1:-prof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/stats.log 2>&1 || { echo stats_failed; tail -20 $OUT/stats.log; exit 1; }
echo stats_ok
# kernel-family breakdown: graph replays only (no roofline-timing steps, whose conv launches repeat 4x)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/steps -o run -- python bench.py --steps 10 --warmup 2 --roofline-steps 0 --no-cpu-baseline > $OUT/steps.log 2>&1 || { echo steps_failed; tail -20 $OUT/steps.log; exit 1; }
python scripts/kernel_breakdown.py $OUT/steps/run_kernel_stats.csv > $OUT/breakdown.md
echo steps_ok
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python bench.py --no-graph --steps 2 --warmup 1 --roofline-steps 1 --no-cpu-baseline > $OUT/pmc_fetch.log 2>&1 || { echo fetch_failed; tail -20 $OUT/pmc_fetch.log; exit 1; }
echo fetch_ok
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python bench.py --no-graph --steps 2 --warmup 1 --roofline-steps 1 --no-cpu-baseline > $OUT/pmc_write.log 2>&1 || { echo write_failed; tail -20 $OUT/pmc_write.log; exit 1; }
echo write_ok
python scripts/pmc_traffic.py $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_traffic.json && cp $OUT/pmc_traffic.json profiles/pmc_traffic.json
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1 || { echo bench_failed; tail -30 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json; cut -c1-600 $OUT/bench.json
