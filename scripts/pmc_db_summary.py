"""Mean counter values per kernel from rocprofv3 --pmc output directories (rocpd sqlite .db files).
usage: python scripts/pmc_db_summary.py <kernel-name substring> <dir> [<dir> ...]"""
import collections, glob, sqlite3, sys

pat = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
meta = {}
for d in sys.argv[2:]:
    for fn in glob.glob(f"{d}/**/*.db", recursive=True):
        c = sqlite3.connect(fn)
        q = ("select kernel_name, counter_name, value, vgpr_count, lds_block_size, grid_size from counters_collection")
        for kn, cn, v, vg, lds, gs in c.execute(q):
            if pat in kn and v is not None:
                agg[kn[:70]][cn].append(float(v))
                meta[kn[:70]] = (vg, lds, gs)
for k, d in agg.items():
    print(k, "vgpr/lds/grid", meta[k])
    for cn, v in sorted(d.items()):
        print(f"   {cn:28s} {sum(v) / len(v):16.0f}  (n={len(v)})")
