# TSSA at 512 threads as the default: packed-head / block / grads tests, l-scale A/B against the 256-thread build
mkdir -p gpurun_out/r06bw
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_packed_head.py tests/test_gpu_blocks.py tests/test_gpu_grads.py tests/test_gpu_net.py 2>&1 | tail -1
for L in ab/tssa256.so yolo-ad-refine_amd/adrefine/lib/libadr_hip.so ab/tssa256.so yolo-ad-refine_amd/adrefine/lib/libadr_hip.so; do
  ADR_LIB=$L timeout -k 10 300 python -u bench.py --scale l --img 1280 --bs 16 --steps 8 --warmup 3 --roofline-steps 0 --stage-check 0 --no-cpu-baseline --infer-steps 0 --augment-bench 0 > gpurun_out/r06bw/l.log 2>&1 || exit 1
  echo "$L $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r06bw/l.log | head -1)"
done
