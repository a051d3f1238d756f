# A/B the bf16 conv engine: new (in-tree) vs old (adrefine/lib/old) library on the representative shapes.
set -o pipefail
for lib in new old; do
  if [ $lib = old ]; then export ADR_LIB=$PWD/yolo-ad-refine_amd/adrefine/lib/old/libadr_hip.so ADR_HEADER=$PWD/yolo-ad-refine_amd/adrefine/lib/old/adr.h; fi
  echo "== $lib"
  MODES="${MODES:-fwd2 dgrad2}" bash scripts/conv_shapes.sh 2>&1 | grep -v amdgpu.ids || exit 1
done
