# TSSA kernels with 1024-thread blocks: model-level parity tests, n- and l-scale A/B against the HEAD build
mkdir -p gpurun_out/r06aj
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
NEW=yolo-ad-refine_amd/adrefine/lib/libadr_hip.so
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_blocks.py tests/test_gpu_net.py tests/test_gpu_grads.py tests/test_gpu_bf16.py > gpurun_out/r06aj/tests.log 2>&1 || { tail -30 gpurun_out/r06aj/tests.log; exit 1; }; tail -1 gpurun_out/r06aj/tests.log &&
bash scripts/ab_lib.sh gpurun_out/r06aj/n.txt "python bench.py --no-cpu-baseline --steps 40 --infer-steps 0 --roofline-steps 0 --stage-check 0 --augment-bench 0 --lscale-steps 0" ab/head.so $NEW 2 &&
grep -o '"ms_per_step": [0-9.]*\|== .*' gpurun_out/r06aj/n.txt &&
for L in ab/head.so $NEW ab/head.so $NEW; do
  ADR_LIB=$L timeout -k 10 300 python -u bench.py --scale l --img 1280 --bs 16 --steps 8 --warmup 3 --roofline-steps 0 --stage-check 0 --no-cpu-baseline --infer-steps 0 --augment-bench 0 > gpurun_out/r06aj/l.log 2>&1 || exit 1
  echo "$L $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r06aj/l.log)"
done
