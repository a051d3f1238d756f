# dcn_bwd phase A/B at the n-scale P3 shape: mode bits 1 / 2 skip a phase, 4 disables the zero-K-step skip
set -o pipefail
for m in 0 4 1 5 2; do ADR_DCN_BWD_MODE=$m timeout -k 10 60 python scripts/dcn_bwd_micro.py 2>&1 | grep dcn_bwd || exit 1; done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/dcnpmc2; mkdir -p $OUT
for m in 1 2; do
export ADR_DCN_BWD_MODE=$m
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAIT_ANY SQ_INSTS_VMEM_RD --output-format csv -d $OUT/p1_$m -o run -- python3 scripts/dcn_bwd_micro.py > $OUT/p1_$m.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_WAVES SQ_INST_CYCLES_VMEM --output-format csv -d $OUT/p2_$m -o run -- python3 scripts/dcn_bwd_micro.py > $OUT/p2_$m.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob, collections
for d in sorted(glob.glob("gpurun_out/dcnpmc2/p*_*")):
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    if not f: continue
    acc = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f[0])):
        if "dcn_bwd_kernel" not in r["Kernel_Name"]: continue
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(d, {k: round(v / max(1, n[k]) / 1e6, 3) for k, v in acc.items()}, "(M per launch)")
PY
