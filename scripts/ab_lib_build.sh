#!/bin/bash
# Build an A/B variant of libadr_hip.so (CPU): the named csrc files taken from git revision REV, every other object
# from the current in-tree build. usage: bash scripts/ab_lib_build.sh NAME REV file.hip [file.hip ...]
# -> ab/NAME.so (load it with ADR_LIB=ab/NAME.so)
set -e
NAME=$1; REV=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/yolo-ad-refine_amd
make -s -C "$PKG" -j8
T=$(mktemp -d)
mkdir -p "$T/pkg/csrc" "$T/include"
cp "$PKG"/csrc/*.h "$T/pkg/csrc/"
cp "$ROOT"/include/*.h "$T/include/"
OBJS=""
for o in "$PKG"/build/obj/*.o; do
  b=$(basename "$o" .o)
  skip=0
  for f in "$@"; do [ "$(basename "$f" .hip)" = "$b" ] && skip=1; done
  [ $skip = 1 ] || OBJS="$OBJS $o"
done
for f in "$@"; do
  git -C "$ROOT" show "$REV:yolo-ad-refine_amd/csrc/$f" > "$T/pkg/csrc/$f"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -c "$T/pkg/csrc/$f" -o "$T/${f%.hip}.o"
  OBJS="$OBJS $T/${f%.hip}.o"
done
mkdir -p "$ROOT/ab"
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o "$ROOT/ab/$NAME.so" $OBJS
rm -rf "$T"
echo "ab/$NAME.so"
