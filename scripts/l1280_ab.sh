# same-box A/B of environment settings on configs[4] (l-scale, 1280^2, bs 16; short runs, no CPU / inference legs)
# usage: bash scripts/l1280_ab.sh <tag> "<envA>" "<envB>" ["<envC>"]
set -o pipefail
TAG=$1; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT
i=0
for E in "$@"; do
  i=$((i+1))
  env $E timeout -k 10 300 python -u bench.py --scale l --img 1280 --bs 16 --steps 8 --warmup 3 --roofline-steps 0 \
    --stage-check 0 --no-cpu-baseline --infer-steps 0 --augment-bench 0 > $OUT/r$i.log 2>&1 || { tail -5 $OUT/r$i.log; exit 1; }
  echo "[$E] $(grep -o '"ms_per_step": [0-9.]*' $OUT/r$i.log)"
done
