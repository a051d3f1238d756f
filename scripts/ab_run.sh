set -o pipefail
mkdir -p gpurun_out
for lib in new old; do
  if [ $lib = old ]; then export ADR_LIB=$PWD/yolo-ad-refine_amd/adrefine/lib/old/libadr_hip.so ADR_HEADER=$PWD/yolo-ad-refine_amd/adrefine/lib/old/adr.h; fi
  echo "== $lib"
  timeout -k 10 120 python scripts/ab_block.py ayhead || exit 1
done
unset ADR_LIB ADR_HEADER
timeout -k 10 300 python -m pytest tests/test_gpu_nms.py -q -p no:cacheprovider 2>&1 | tail -5
