# Round-6 measurement set on one box (usage: bash scripts/profile_r06.sh <tag>):
#   1. PMC calibration per access pattern (scripts/pmc_calibrate.py; FETCH and WRITE passes)
#   2. per-kernel HBM bytes per launch: FETCH / WRITE passes over eager bench steps -> profiles/pmc_traffic.json
#   3. rocprofv3 --kernel-trace --stats of a graph-replayed bench run -> replay table + whole-step traffic
#   4. the default bench line (with cpu_baseline, inference, l-scale object) reading 2-3's outputs
set -o pipefail
TAG=${1:-r06}
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/cal_fetch -o run -- python3 scripts/pmc_calibrate.py run $OUT/cal > $OUT/cal_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/cal_write -o run -- python3 scripts/pmc_calibrate.py run $OUT/cal > $OUT/cal_write.log 2>&1 &&
python3 scripts/pmc_calibrate.py combine $OUT/cal_fetch $OUT/cal_write $OUT/cal/known.json $OUT/pmc_calibration.json > $OUT/cal.log 2>&1 || { tail -20 $OUT/cal*.log; exit 1; }
bash scripts/pmc_bench_traffic.sh || exit 1
cp gpurun_out/pmc_bench/pmc_traffic.json profiles/pmc_traffic.json && cp gpurun_out/pmc_bench/pmc_traffic.json $OUT/ || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 25 --warmup 2 --no-cpu-baseline --infer-steps 0 --augment-bench 0 --lscale-steps 0 --stage-check 0 --roofline-steps 0 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
TRACE=$(find $OUT/prof -name "*kernel_trace.csv" | head -1)
python3 scripts/replay_breakdown.py $TRACE --steps 8 --top 40 --pmc profiles/pmc_traffic.json > $OUT/replay.md 2>&1 || exit 1
python3 scripts/step_traffic.py $TRACE profiles/pmc_traffic.json $OUT/step_traffic.json --bs 64 > $OUT/step_traffic.log 2>&1 || { cat $OUT/step_traffic.log; exit 1; }
cp $OUT/step_traffic.json profiles/step_traffic.json || exit 1
timeout -k 10 600 python3 bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json
echo done
