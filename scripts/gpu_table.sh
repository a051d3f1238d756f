set -o pipefail
OUT=gpurun_out/${1:-table}; mkdir -p $OUT
timeout -k 10 300 python scripts/conv_table.py > $OUT/conv_table.txt 2>&1; echo rc=$?; head -70 $OUT/conv_table.txt
