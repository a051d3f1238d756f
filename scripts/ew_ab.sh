# A/B of the adr_ew grid cap (ADR_EW_BLOCKS, 0 = the old 32768 cap)
set -o pipefail
OUT=gpurun_out/${1:-ew}; mkdir -p $OUT
for cap in 0 2048 4096 1024; do
  echo "== ADR_EW_BLOCKS=$cap" >> $OUT/micro.txt
  ADR_EW_BLOCKS=$cap timeout -k 10 120 python scripts/norm_micro.py >> $OUT/micro.txt 2>&1 || exit 1
done
