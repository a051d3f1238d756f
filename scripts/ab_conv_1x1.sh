# 1x1 / wide-K conv shapes of the step: this tree's library vs abtree/'s
set -e
OLD=abtree/yolo-ad-refine_amd/adrefine/lib/libadr_hip.so
while read -r m args; do
  echo -n "new "; timeout -k 5 60 python scripts/conv_micro.py $m $args 2>/dev/null
  echo -n "old "; ADR_LIB=$OLD ADR_HEADER=abtree/include/adr.h timeout -k 5 60 python scripts/conv_micro.py $m $args 2>/dev/null
done <<'SHAPES'
fwd2 64 80 80 128 128 1 1 1
fwd2 64 80 80 64 576 1 1 1
fwd2 64 40 40 256 128 1 1 1
fwd2 64 20 20 256 128 1 1 1
fwd2 64 80 80 192 128 1 1 1
dgrad2 64 80 80 128 128 1 1 1
dgrad2 64 80 80 128 192 1 1 1
dgrad2 64 40 40 128 192 1 1 1
fwd2 64 80 80 128 128 3 3 2
SHAPES
