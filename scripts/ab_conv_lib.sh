# conv micro A/B: this tree's library vs abtree/'s (scripts/ab_snapshot.sh), same shapes, alternating
set -e
OLD=abtree/yolo-ad-refine_amd/adrefine/lib/libadr_hip.so
while read -r m args; do
  echo -n "new "; timeout -k 5 60 python scripts/conv_micro.py $m $args 2>/dev/null
  echo -n "old "; ADR_LIB=$OLD ADR_HEADER=abtree/include/adr.h timeout -k 5 60 python scripts/conv_micro.py $m $args 2>/dev/null
done <<'SHAPES'
fwd2 64 80 80 64 64 3 3 1
fwd2 64 40 40 128 128 3 3 1
fwd2 64 80 80 128 64 1 1 1
fwd2 64 40 40 64 128 1 1 1
fwd2 64 160 160 32 64 3 3 2
dgrad2 64 80 80 64 64 3 3 1
dgrad2 64 40 40 128 128 3 3 1
dgrad2 64 80 80 128 64 1 1 1
dgrad2 64 160 160 32 64 3 3 2
wgrad 64 80 80 64 64 3 3 1
wgrad 64 80 80 128 128 3 3 2
wgrad 64 320 320 16 32 3 3 2
wgrad 64 40 40 128 128 1 1 1
wgrad 64 80 80 64 32 3 3 1
SHAPES
