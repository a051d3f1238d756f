# A/B the bench: current tree vs the snapshot in abtree/ (another commit's package + library), alternating runs
set -o pipefail
for i in 1 2; do
  echo -n "new: "; timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' || exit 1
  echo -n "old: "; (cd abtree && timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 2>/dev/null | grep -o '"ms_per_step": [0-9.]*') || exit 1
done
