#!/bin/bash
# Same-box A/B of library builds (GPU box): bash scripts/ab_lib.sh OUT "<command>" libA libB [reps]
# runs <command> with ADR_LIB=libX alternately, `reps` times each; appends each run's output to OUT
set -o pipefail
OUT=$1; CMD=$2; A=$3; B=$4; R=${5:-2}
for r in $(seq 1 $R); do
  for L in $A $B; do
    echo "== $L run $r" >> $OUT
    ADR_LIB=$L timeout -k 10 120 bash -c "$CMD" >> $OUT 2>&1 || { echo "FAILED $L"; exit 1; }
  done
done
