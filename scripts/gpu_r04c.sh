# r04c: configs[4] (l-scale, 1280^2, bs 16): the wide 3x3 tile on / off, the fp8 forward convs, a kernel profile,
# and the per-shape fp8 micro-benchmark
set -o pipefail
OUT=gpurun_out/r04c; mkdir -p $OUT
lb() {  # label, extra args, env...
  local label=$1 extra=$2; shift 2
  env "$@" timeout -k 10 400 python -u bench.py --scale l --img 1280 --bs 16 --steps 10 --warmup 3 --roofline-steps 0 \
      --stage-check 0 $extra > $OUT/$label.log 2>&1 || { echo "$label FAIL"; tail -20 $OUT/$label.log; return 1; }
  grep '^{' $OUT/$label.log | tail -1 > $OUT/$label.json
  python -c "import json;d=json.load(open('$OUT/$label.json'));print('$label', d['ms_per_step'], d['value'], d['dtype'], d['peak_hbm_gib'], d['host_enqueue_ms_per_step'])"
}
lb wide "" ADR_CONV3W=1 && lb narrow "" ADR_CONV3W=0 && lb wide_fp8 "--conv-fp8" ADR_CONV3W=1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --scale l \
    --img 1280 --bs 16 --steps 3 --warmup 2 --roofline-steps 0 --stage-check 0 > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 1; }
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cp $f $OUT/kernel_stats.csv
python3 scripts/kernel_breakdown.py $OUT/kernel_stats.csv
timeout -k 10 300 python scripts/fp8_micro.py > $OUT/fp8_micro.txt 2>&1; cat $OUT/fp8_micro.txt
