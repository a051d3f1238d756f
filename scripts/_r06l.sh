# staged-step overhead on one GPU by DDP bucket size (the one-rank RCCL group included)
mkdir -p gpurun_out/r06l
for mb in 4 8 16; do
  ADR_DDP_BUCKET_MB=$mb timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --infer-steps 0 \
    --augment-bench 0 --lscale-steps 0 --roofline-steps 0 > gpurun_out/r06l/b$mb.log 2>&1 || exit 1
  echo "bucket $mb MB: $(grep '^{' gpurun_out/r06l/b$mb.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["ddp_staging"]; print(s["cuts"], s["ms_per_step_unstaged"], s["ms_per_step_staged"], s["ms_per_step_staged_rccl"], s["rccl_overhead_vs_unstaged"])')" >> gpurun_out/r06l/summary.txt
done
