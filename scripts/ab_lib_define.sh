#!/bin/bash
# Build an A/B variant of libadr_hip.so (CPU) with extra -D flags for the named csrc files, every other object from
# the current in-tree build: bash scripts/ab_lib_define.sh NAME "-DFOO=0" file.hip [file.hip ...] -> ab/NAME.so
set -e
NAME=$1; DEFS=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/yolo-ad-refine_amd
make -s -C "$PKG" -j8
T=$(mktemp -d)
OBJS=""
for o in "$PKG"/build/obj/*.o; do
  b=$(basename "$o" .o)
  skip=0
  for f in "$@"; do [ "$(basename "$f" .hip)" = "$b" ] && skip=1; done
  [ $skip = 1 ] || OBJS="$OBJS $o"
done
for f in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $DEFS -c "$PKG/csrc/$f" -o "$T/${f%.hip}.o"
  OBJS="$OBJS $T/${f%.hip}.o"
done
mkdir -p "$ROOT/ab"
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o "$ROOT/ab/$NAME.so" $OBJS
rm -rf "$T"
echo "ab/$NAME.so"
