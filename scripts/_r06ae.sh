# bijective XCD remap (every grid size) + per-entry remap in the batched WGRAD: bitwise check, DCN tests / micro / L2 hits,
# n- and l-scale A/B against the HEAD build (ab/head.so)
mkdir -p gpurun_out/r06ae
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
NEW=yolo-ad-refine_amd/adrefine/lib/libadr_hip.so
timeout -k 10 120 python3 scripts/wgrad_db_check.py > gpurun_out/r06ae/db.txt 2>&1 && tail -1 gpurun_out/r06ae/db.txt &&
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu tests/test_gpu_dcn.py tests/test_gpu_wgrad_bias.py tests/test_gpu_defer.py > gpurun_out/r06ae/tests.log 2>&1 || { tail -30 gpurun_out/r06ae/tests.log; exit 1; }; tail -1 gpurun_out/r06ae/tests.log &&
for L in ab/head.so $NEW; do ADR_LIB=$L R=10 timeout -k 10 90 python3 scripts/dcn_wgrad_levels_micro.py 2>&1 | grep -v amdgpu; done &&
R=3 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum --output-format csv -d gpurun_out/r06ae/p1 -o run -- python3 scripts/dcn_wgrad_levels_micro.py > gpurun_out/r06ae/p1.log 2>&1 &&
bash scripts/ab_lib.sh gpurun_out/r06ae/n.txt "python bench.py --no-cpu-baseline --steps 40 --infer-steps 0 --roofline-steps 0 --stage-check 0 --augment-bench 0 --lscale-steps 0" ab/head.so $NEW 3 &&
grep -o '"ms_per_step": [0-9.]*\|== .*' gpurun_out/r06ae/n.txt &&
for L in ab/head.so $NEW ab/head.so $NEW; do
  ADR_LIB=$L timeout -k 10 300 python -u bench.py --scale l --img 1280 --bs 16 --steps 8 --warmup 3 --roofline-steps 0 --stage-check 0 --no-cpu-baseline --infer-steps 0 --augment-bench 0 > gpurun_out/r06ae/l.log 2>&1 || exit 1
  echo "$L $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r06ae/l.log)"
done
