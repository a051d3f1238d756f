set -o pipefail
OUT=gpurun_out/dcnprof; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/n -o run -- python3 scripts/dcn_bench.py > $OUT/n.log 2>&1 && \
N=16 C=256 SIZES=160,80,40 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/l -o run -- python3 scripts/dcn_bench.py > $OUT/l.log 2>&1
rc=$?
for d in n l; do f=$(find $OUT/$d -name "*kernel_stats.csv" | head -1); echo "== $d"; python3 -c "
import csv,sys
for r in list(csv.DictReader(open('$f')))[:12]: print(f\"{float(r['AverageNs'])/1e3:9.1f}us x{r['Calls']:>5} {r['Name'][:90]}\")"; done
exit $rc
