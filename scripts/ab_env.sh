# A/B one environment knob on the current tree: bash scripts/ab_env.sh VAR "val1 val2 ..."
set -o pipefail
VAR=$1
for i in 1 2; do
  for v in $2; do
    echo -n "$VAR=$v: "; env $VAR=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' || exit 1
  done
done
