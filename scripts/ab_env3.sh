# Same-box A/B/C.. of environment settings on the bench step: bash scripts/ab_env3.sh <tag> <reps> "<envA>" "<envB>" ["<envC>" ...]
# (settings run alternately, `reps` rounds; prints ms_per_step per run)
set -o pipefail
TAG=$1; R=$2; shift 2; OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in $(seq 1 $R); do
  i=0
  for E in "$@"; do
    i=$((i+1))
    env $E timeout -k 10 240 python bench.py --no-cpu-baseline --steps 30 --infer-steps 0 --roofline-steps 0 > $OUT/v$i.$r.log 2>&1 || { tail -5 $OUT/v$i.$r.log; exit 1; }
    echo "v$i [$E] run $r: $(grep -o '"ms_per_step": [0-9.]*' $OUT/v$i.$r.log)"
  done
done
