set -e
for i in 1 2; do
echo -n "new "; timeout -k 5 60 python scripts/dcn_micro.py 2>/dev/null
echo -n "old "; ADR_LIB=abtree/yolo-ad-refine_amd/adrefine/lib/libadr_hip.so ADR_HEADER=abtree/include/adr.h timeout -k 5 60 python scripts/dcn_micro.py 2>/dev/null
done
