# A/B of the streaming-kernel launch shape: grid cap (ADR_STREAM_BLOCKS, 0 = uncapped) and nc_reduce chunk rows.
set -o pipefail
OUT=gpurun_out/${1:-nm}; mkdir -p $OUT
for cfg in "0 256" "2048 256" "1024 256" "4096 256" "2048 512" "2048 1024"; do
  set -- $cfg
  echo "== ADR_STREAM_BLOCKS=$1 ADR_NC_ROWS=$2" >> $OUT/micro.txt
  ADR_STREAM_BLOCKS=$1 ADR_NC_ROWS=$2 timeout -k 10 120 python scripts/norm_micro.py >> $OUT/micro.txt 2>&1 || exit 1
done
