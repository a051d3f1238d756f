# representative conv contractions of the n/640 bs64 step; MODES overrides the list
set -e
MODES=${MODES:-"fwd fwd2 dgrad dgrad2"}
for m in $MODES; do
  timeout -k 5 60 python scripts/conv_micro.py $m 64 80 80 64 64 3 3 1
  timeout -k 5 60 python scripts/conv_micro.py $m 64 80 80 128 128 1 1 1
  timeout -k 5 60 python scripts/conv_micro.py $m 64 80 80 128 128 3 3 2
  timeout -k 5 60 python scripts/conv_micro.py $m 64 20 20 128 128 1 1 1
  timeout -k 5 60 python scripts/conv_micro.py $m 64 640 640 8 16 3 3 2
  timeout -k 5 60 python scripts/conv_micro.py $m 64 160 160 16 8 3 3 1
  timeout -k 5 60 python scripts/conv_micro.py $m 64 80 80 64 576 1 1 1
  timeout -k 5 60 python scripts/conv_micro.py $m 64 40 40 128 256 3 3 2
done
