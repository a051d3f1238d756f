# TSSA loads in flight per thread (TSSA_LOADS 2 / 4 / 8 at 512 threads): l-scale 2 runs each, n-scale 3 runs each
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 1 2; do for L in yolo-ad-refine_amd/adrefine/lib/libadr_hip.so ab/tssa_u8.so ab/tssa_u2.so; do
  ADR_LIB=$L timeout -k 10 300 python -u bench.py --scale l --img 1280 --bs 16 --steps 8 --warmup 3 --roofline-steps 0 --stage-check 0 --no-cpu-baseline --infer-steps 0 --augment-bench 0 > gpurun_out/l.log 2>&1 || exit 1
  echo "l $L $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/l.log | head -1)"
done; done
for r in 1 2 3; do for L in yolo-ad-refine_amd/adrefine/lib/libadr_hip.so ab/tssa_u8.so ab/tssa_u2.so; do
  ADR_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 --infer-steps 0 --roofline-steps 0 --stage-check 0 --augment-bench 0 --lscale-steps 0 > gpurun_out/n.log 2>&1 || exit 1
  echo "n $L $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/n.log | head -1)"
done; done
