# HBM traffic per kernel of the bench step: two separate rocprofv3 --pmc passes (FETCH_SIZE; WRITE_SIZE) over
# an eager bench run, combined by scripts/pmc_traffic.py into profiles/pmc_traffic.json (gfx950 corrections there).
set -o pipefail
OUT=gpurun_out/pmc_bench; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
CMD="python3 bench.py --no-graph --steps 2 --warmup 1 --roofline-steps 0 --no-cpu-baseline --infer-steps 0 --stage-check 0 --augment-bench 0 --lscale-steps 0"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $CMD > $OUT/fetch.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $CMD > $OUT/write.log 2>&1 &&
python3 scripts/pmc_traffic.py $OUT/fetch $OUT/write $OUT/pmc_traffic.json
