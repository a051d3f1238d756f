# WGRAD split-K partial budget A/B on the whole step (ADR_WG_PART_MB; default 24)
set -o pipefail
OUT=gpurun_out/wgab; mkdir -p $OUT
for mb in 24 48 96 24 48 96; do ADR_WG_PART_MB=$mb timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 --warmup 10 --infer-steps 0 --stage-check 0 --augment-bench 0 --roofline-steps 0 > $OUT/b$mb.log 2>&1 || { tail $OUT/b$mb.log; exit 1; }
python -c "import json;d=[json.loads(l) for l in open('$OUT/b$mb.log') if l.startswith('{')][-1];print('part_mb=$mb', d['ms_per_step'], d['ms_per_step_events']['median'])"; done
