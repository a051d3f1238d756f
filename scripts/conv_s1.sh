# generic (fwd/dgrad) vs bf16 engine (fwd2/dgrad2) on the stride-1 multi-tap shapes of the n/640 bs64 step
set -e
for m in fwd fwd2 dgrad dgrad2; do
  timeout -k 5 60 python scripts/conv_micro.py $m 64 80 80 64 64 3 3 1
  timeout -k 5 60 python scripts/conv_micro.py $m 64 80 80 128 64 3 3 1
  timeout -k 5 60 python scripts/conv_micro.py $m 64 40 40 64 64 3 3 1
  timeout -k 5 60 python scripts/conv_micro.py $m 64 40 40 128 128 3 3 1
  timeout -k 5 60 python scripts/conv_micro.py $m 64 20 20 64 64 3 3 1
  timeout -k 5 60 python scripts/conv_micro.py $m 64 20 20 128 128 3 3 1
  timeout -k 5 60 python scripts/conv_micro.py $m 64 160 160 64 64 3 3 1
done
