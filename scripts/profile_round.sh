# Refresh the committed measurement set on one box (usage: bash scripts/profile_round.sh <tag>):
#   1. HBM traffic per kernel: two rocprofv3 --pmc passes (FETCH_SIZE; WRITE_SIZE) -> pmc_traffic.json, installed
#      as profiles/pmc_traffic.json on the box so the bench line's roofline.traffic uses it
#   2. the default bench line (1 GPU, with cpu_baseline and the inference summary)
#   3. the configs[1] inference line (bench.py --infer)
#   4. rocprofv3 --kernel-trace --stats of a 25-step bench run
set -o pipefail
TAG=${1:-r}
OUT=gpurun_out/$TAG; mkdir -p $OUT
bash scripts/pmc_bench_traffic.sh || exit 1
cp gpurun_out/pmc_bench/pmc_traffic.json profiles/pmc_traffic.json && cp gpurun_out/pmc_bench/pmc_traffic.json $OUT/ || exit 1
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json
timeout -k 10 300 python bench.py --infer --steps 20 --warmup 2 > $OUT/infer.log 2>&1 || { tail -20 $OUT/infer.log; exit 1; }
grep '^{' $OUT/infer.log | tail -1 > $OUT/infer.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 25 --warmup 2 --no-cpu-baseline --infer-steps 0 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv"
