# Same-box sweep of environment settings against the default, interleaved: bash scripts/ab_sweep.sh <tag> reps "<env1>" "<env2>" ...
# (the default runs before every setting; prints ms_per_step per run)
set -o pipefail
TAG=$1; R=$2; shift 2; OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in $(seq 1 $R); do
  for E in "ADR_NONE=0" "$@"; do
    env $E timeout -k 10 240 python bench.py --no-cpu-baseline --steps 30 --infer-steps 0 --roofline-steps 0 --stage-check 0 --augment-bench 0 --lscale-steps 0 > $OUT/run.log 2>&1 || { tail -5 $OUT/run.log; exit 1; }
    echo "[$E] run $r: $(grep -o '"ms_per_step": [0-9.]*' $OUT/run.log)"
  done
done
