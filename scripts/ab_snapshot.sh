# Snapshot a commit (default HEAD) into abtree/ for scripts/ab_bench.sh: its package sources plus a library
# built from those sources (built here on the CPU host, in abtree/).
set -e
rev=${1:-HEAD}
rm -rf abtree && mkdir abtree
git archive "$rev" bench.py yolo-ad-refine_amd include tests/configs | tar -x -C abtree
make -C abtree/yolo-ad-refine_amd -j8 > /dev/null
ls -la abtree/yolo-ad-refine_amd/adrefine/lib/libadr_hip.so
