# l-scale (configs[4]) same-box sweep of environment settings against the default, interleaved:
# bash scripts/ab_sweep_l.sh <tag> reps "<env1>" ...
set -o pipefail
TAG=$1; R=$2; shift 2; OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in $(seq 1 $R); do
  for E in "ADR_NONE=0" "$@"; do
    env $E timeout -k 10 300 python -u bench.py --scale l --img 1280 --bs 16 --steps 8 --warmup 3 --roofline-steps 0 --stage-check 0 --no-cpu-baseline --infer-steps 0 --augment-bench 0 > $OUT/run.log 2>&1 || { tail -5 $OUT/run.log; exit 1; }
    echo "[$E] run $r: $(grep -o '"ms_per_step": [0-9.]*' $OUT/run.log | head -1)"
  done
done
