# A/B: the streaming 1x1 kernel for forward convs with 129-256 reduction channels on large maps (ADR_C1F256 = min rows)
set -o pipefail
OUT=gpurun_out/ab_c1; mkdir -p $OUT
for v in 0 100000 0 100000; do
  ADR_C1F256=$v timeout -k 10 300 python -u bench.py --scale l --img 1280 --bs 16 --steps 10 --warmup 3 --roofline-steps 0 \
    --stage-check 0 --no-cpu-baseline --infer-steps 0 --augment-bench 0 > $OUT/l_$v.log 2>&1 || { tail -20 $OUT/l_$v.log; exit 1; }
  python -c "import json;a=[json.loads(l) for l in open('$OUT/l_$v.log') if l.startswith('{')][-1];print('l $v',a['ms_per_step'])"
done
for v in 0 100000; do
  ADR_C1F256=$v timeout -k 10 300 python -u bench.py --steps 40 --warmup 10 --no-cpu-baseline --infer-steps 0 --stage-check 0 \
    --augment-bench 0 --roofline-steps 0 > $OUT/n_$v.log 2>&1 || { tail -20 $OUT/n_$v.log; exit 1; }
  python -c "import json;a=[json.loads(l) for l in open('$OUT/n_$v.log') if l.startswith('{')][-1];print('n $v',a['ms_per_step'])"
done
