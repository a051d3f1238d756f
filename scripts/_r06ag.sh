# DCN: weight gradient with all output channels per block (COT = Cout), forward with 128-wide output tiles
# (Cout % 128 == 0): tests, micro (n- and l-scale widths), l-scale and n-scale A/B against the HEAD build
mkdir -p gpurun_out/r06ag
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
NEW=yolo-ad-refine_amd/adrefine/lib/libadr_hip.so
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu tests/test_gpu_dcn.py tests/test_gpu_lscale.py tests/test_gpu_packed_head.py > gpurun_out/r06ag/tests.log 2>&1 || { tail -30 gpurun_out/r06ag/tests.log; exit 1; }; tail -1 gpurun_out/r06ag/tests.log &&
for L in ab/head.so $NEW; do ADR_LIB=$L N=16 C=256 S=160 R=5 timeout -k 10 90 python3 scripts/dcn_wgrad_levels_micro.py 2>&1 | grep -v amdgpu || exit 1; done &&
for L in ab/head.so $NEW; do ADR_LIB=$L N=16 C=256 SIZES=160,80,40 timeout -k 10 120 python3 scripts/dcn_bench.py 2>&1 | grep -v amdgpu || exit 1; done &&
for L in ab/head.so $NEW ab/head.so $NEW; do
  ADR_LIB=$L timeout -k 10 300 python -u bench.py --scale l --img 1280 --bs 16 --steps 8 --warmup 3 --roofline-steps 0 --stage-check 0 --no-cpu-baseline --infer-steps 0 --augment-bench 0 > gpurun_out/r06ag/l.log 2>&1 || exit 1
  echo "$L $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r06ag/l.log)"
done
