# depthwise kernels in isolation: kernel-trace stats, then one PMC pass (wave state breakdown)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05dw; mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 scripts/dw_micro.py > $O/kt.log 2>&1 || exit 1
tail -5 $O/kt.log
true
python3 - <<'P'
import csv, glob, collections
f = glob.glob('gpurun_out/r05dw/kt/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'dw' in r['Name']: print(r['Name'][:70], r['Calls'], r['AverageNs'])
f = glob.glob('gpurun_out/r05dw/pmc/**/*counter_collection.csv', recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r['Kernel_Name'][:60]
    if 'dw' not in k: continue
    acc[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, d in acc.items():
    print(k, {c: round(v / 1e3, 1) for c, v in sorted(d.items())})
P
