# stem kernels: micro timing + one SQ PMC pass (where do the waves wait)
mkdir -p gpurun_out/r06bb
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u scripts/stem_micro.py 64 640 16 20 > gpurun_out/r06bb/micro.txt 2>&1 || { tail -20 gpurun_out/r06bb/micro.txt; exit 1; }
cat gpurun_out/r06bb/micro.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -d gpurun_out/r06bb/pmc -o pmc -- python3 scripts/stem_micro.py 64 640 16 2 > gpurun_out/r06bb/pmc.log 2>&1 || { tail -20 gpurun_out/r06bb/pmc.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/r06bb/pmc/**/*counter_collection.csv", recursive=True)
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for fn in f:
    for r in csv.DictReader(open(fn)):
        if "stem" in r["Kernel_Name"]:
            agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY
