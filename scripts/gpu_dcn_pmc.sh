#!/bin/bash
# DCN backward stall breakdown (one --pmc pass per mode). usage (GPU box): bash scripts/gpu_dcn_pmc.sh OUTDIR
set -e
out=${1:-gpurun_out/dcn_pmc}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
for m in 0 1 2; do
  ADR_DCN_BWD_MODE=$m R=5 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU -d "$out/m$m" -o pmc --output-format csv \
    -- python3 scripts/dcn_bwd_micro.py
done
python3 - "$out" <<'PY'
import csv, glob, sys, collections
for m in (0, 1, 2):
    tot = collections.defaultdict(float); n = collections.Counter()
    for f in glob.glob(f"{sys.argv[1]}/m{m}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "dcn_bwd" not in r["Kernel_Name"]:
                continue
            tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(f"mode {m}: " + "  ".join(f"{k}={tot[k]/max(n[k],1):.3g}" for k in sorted(tot)))
PY
