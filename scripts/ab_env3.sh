# Same-box A/B of environment settings on the bench step (fast form: no side legs):
#   bash scripts/ab_env3.sh <tag> "<envA>" "<envB>" [reps]   (alternating runs; prints ms_per_step per run)
set -o pipefail
TAG=$1; A=$2; B=$3; R=${4:-2}; OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in $(seq 1 $R); do
  for v in A B; do
    E=$([ $v = A ] && echo "$A" || echo "$B")
    env $E timeout -k 10 240 python bench.py --no-cpu-baseline --steps 40 --infer-steps 0 --roofline-steps 0 \
      --stage-check 0 --augment-bench 0 --lscale-steps 0 > $OUT/$v$r.log 2>&1 || { tail -5 $OUT/$v$r.log; exit 1; }
    echo "$v [$E] run $r: $(grep -o '"ms_per_step": [0-9.]*' $OUT/$v$r.log)"
  done
done
