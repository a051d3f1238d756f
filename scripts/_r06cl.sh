# DG2H at >= 512 output channels whatever the padding (default now) vs the 15 % padding rule only (ADR_DG2H=1 is
# the default mode; the A/B uses a library built before the change)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_dg2.py tests/test_gpu_conv.py tests/test_gpu_lscale.py 2>&1 | tail -1
for L in ab/pre_dg2.so yolo-ad-refine_amd/adrefine/lib/libadr_hip.so ab/pre_dg2.so yolo-ad-refine_amd/adrefine/lib/libadr_hip.so; do
  ADR_LIB=$L timeout -k 10 300 python -u bench.py --scale l --img 1280 --bs 16 --steps 8 --warmup 3 --roofline-steps 0 --stage-check 0 --no-cpu-baseline --infer-steps 0 --augment-bench 0 > gpurun_out/l.log 2>&1 || exit 1
  echo "$L $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/l.log | head -1)"
done
bash scripts/ab_lib.sh gpurun_out/r06cl_n.txt "python bench.py --no-cpu-baseline --steps 30 --infer-steps 0 --roofline-steps 0 --stage-check 0 --augment-bench 0 --lscale-steps 0" ab/pre_dg2.so yolo-ad-refine_amd/adrefine/lib/libadr_hip.so 2 && grep -o '"ms_per_step": [0-9.]*\|== .*' gpurun_out/r06cl_n.txt
