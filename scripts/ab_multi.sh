# same-box A/B of several environment settings on the bench step: bash scripts/ab_multi.sh <tag> <reps> "<env1>" "<env2>" ...
set -o pipefail
TAG=$1; R=$2; shift 2; OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in $(seq 1 $R); do
  i=0
  for E in "$@"; do
    i=$((i+1))
    env $E timeout -k 10 240 python bench.py --no-cpu-baseline --steps 30 --infer-steps 0 --roofline-steps 0 \
      --stage-check 0 --augment-bench 0 > $OUT/s$i.r$r.log 2>&1 || { tail -5 $OUT/s$i.r$r.log; exit 1; }
    echo "[$E] run $r: $(grep -o '"ms_per_step": [0-9.]*' $OUT/s$i.r$r.log)"
  done
done
