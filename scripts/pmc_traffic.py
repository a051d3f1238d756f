"""HBM traffic per launch from two rocprofv3 --pmc passes (FETCH_SIZE; WRITE_SIZE), per kernel symbol.

  python scripts/pmc_traffic.py <fetch_dir> <write_dir> <out.json>

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts half of the bytes of a 16-byte-per-lane
streaming read, so read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE (KB) is exact for 16-byte stores and float
atomics. Both are memory-side (L2 -> fabric) counts, so Infinity-Cache hits are included. Keys are demangled
kernel names; bench.py demangles its roofline kernel symbol to look them up."""
import csv
import glob
import json
import sys
from collections import defaultdict


def load(d, counter):
    per = defaultdict(dict)  # kernel -> dispatch -> value (summed over the counter's instances)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k, dsp = r["Kernel_Name"], r["Dispatch_Id"]
            per[k][dsp] = per[k].get(dsp, 0.0) + float(r["Counter_Value"])
    return per


def main():
    fdir, wdir, out = sys.argv[1:4]
    fetch, write = load(fdir, "FETCH_SIZE"), load(wdir, "WRITE_SIZE")
    res = {}
    for k in set(fetch) | set(write):
        fv, wv = list(fetch.get(k, {}).values()), list(write.get(k, {}).values())
        if not fv or not wv:
            continue
        rd = 2.0 * 1024.0 * sum(fv) / len(fv)
        wr = 1024.0 * sum(wv) / len(wv)
        res[k] = {"launches": len(fv), "read_bytes_per_launch": round(rd), "write_bytes_per_launch": round(wr),
                  "hbm_bytes_per_launch": round(rd + wr)}
    doc = {"source": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes) over "
                     "`python bench.py --no-graph --steps 2 --warmup 1 --roofline-steps 0 --no-cpu-baseline --infer-steps 0 "
                     "--stage-check 0 --augment-bench 0 --lscale-steps 0` (eager steps only: the replayed step's launch mix); "
                     "read = 2 x FETCH_SIZE x 1 KiB (gfx950 half-count correction), write = WRITE_SIZE x 1 KiB",
           "kernels": dict(sorted(res.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"] * kv[1]["launches"]))}
    json.dump(doc, open(out, "w"), indent=1)
    print(f"{len(res)} kernels -> {out}")


if __name__ == "__main__":
    main()
