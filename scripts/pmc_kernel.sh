# One rocprofv3 --pmc pass over a python command, filtered to kernels matching a regex.
# usage: bash scripts/pmc_kernel.sh <tag> <regex> "<counters>" <python args...>
set -o pipefail
TAG=$1; RX=$2; CNT=$3; shift 3
OUT=gpurun_out/pmc_$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc $CNT --kernel-include-regex "$RX" --output-format csv -d $OUT -o run -- python3 "$@" > $OUT/log.txt 2>&1
rc=$?
f=$(find $OUT -name "*counter_collection.csv" | head -1)
[ -n "$f" ] && python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in rows:
    k = r["Kernel_Name"][:60]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    print(k)
    for c, v in d.items():
        print(f"   {c:28s} {v / n[(k, c)]:.4g} per dispatch")
PY
exit $rc
