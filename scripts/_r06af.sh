# XCD-aware order in the flash attention kernels: micro (n and l shapes), attention parity tests, l- and n-scale A/B
mkdir -p gpurun_out/r06af
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
NEW=yolo-ad-refine_amd/adrefine/lib/libadr_hip.so
for L in ab/head.so $NEW; do
  ADR_LIB=$L timeout -k 10 90 python3 scripts/attn_micro.py 2>&1 | grep -v amdgpu || exit 1
  ADR_LIB=$L B=16 H=4 L=4800 timeout -k 10 90 python3 scripts/attn_micro.py 2>&1 | grep -v amdgpu || exit 1
done &&
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu -k "attn or attention or psa or tssa" tests/ > gpurun_out/r06af/tests.log 2>&1 || { tail -30 gpurun_out/r06af/tests.log; exit 1; }; tail -1 gpurun_out/r06af/tests.log &&
for L in ab/head.so $NEW ab/head.so $NEW; do
  ADR_LIB=$L timeout -k 10 300 python -u bench.py --scale l --img 1280 --bs 16 --steps 8 --warmup 3 --roofline-steps 0 --stage-check 0 --no-cpu-baseline --infer-steps 0 --augment-bench 0 > gpurun_out/r06af/l.log 2>&1 || exit 1
  echo "$L $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r06af/l.log)"
done &&
bash scripts/ab_lib.sh gpurun_out/r06af/n.txt "python bench.py --no-cpu-baseline --steps 40 --infer-steps 0 --roofline-steps 0 --stage-check 0 --augment-bench 0 --lscale-steps 0" ab/head.so $NEW 2 &&
grep -o '"ms_per_step": [0-9.]*\|== .*' gpurun_out/r06af/n.txt
