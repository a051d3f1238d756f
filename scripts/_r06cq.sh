# MLCA attention backward at 512 threads (default now) vs 256: MLCA tests, l-scale 2 runs, n-scale 3 runs each
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_blocks.py tests/test_gpu_grads.py tests/test_gpu_net.py 2>&1 | tail -1
for r in 1 2; do for L in ab/mlca256.so yolo-ad-refine_amd/adrefine/lib/libadr_hip.so; do
  ADR_LIB=$L timeout -k 10 300 python -u bench.py --scale l --img 1280 --bs 16 --steps 8 --warmup 3 --roofline-steps 0 --stage-check 0 --no-cpu-baseline --infer-steps 0 --augment-bench 0 > gpurun_out/l.log 2>&1 || exit 1
  echo "l $L $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/l.log | head -1)"
done; done
for r in 1 2 3; do for L in ab/mlca256.so yolo-ad-refine_amd/adrefine/lib/libadr_hip.so; do
  ADR_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 --infer-steps 0 --roofline-steps 0 --stage-check 0 --augment-bench 0 --lscale-steps 0 > gpurun_out/n.log 2>&1 || exit 1
  echo "n $L $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/n.log | head -1)"
done; done
