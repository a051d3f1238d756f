# conv_bf16 double-buffered tile with straight-line VMEM: micro + n-scale and l-scale library A/B (ab/conv_old.so = HEAD)
mkdir -p gpurun_out/r06z
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
NEW=yolo-ad-refine_amd/adrefine/lib/libadr_hip.so
for L in ab/conv_old.so $NEW; do for sh in "64 80 80 128 128 3 3 2" "16 320 320 256 256 3 3 2" "16 160 160 512 512 3 3 2" "64 40 40 128 256 3 3 2"; do
  ADR_LIB=$L timeout -k 10 60 python3 scripts/conv_micro.py fwd2 $sh 20 >> gpurun_out/r06z/micro_$(basename $L).txt 2>&1 || exit 1
done; done && grep -hv amdgpu.ids gpurun_out/r06z/micro_*.txt &&
bash scripts/ab_lib.sh gpurun_out/r06z/n.txt "python bench.py --no-cpu-baseline --steps 40 --infer-steps 0 --roofline-steps 0 --stage-check 0 --augment-bench 0 --lscale-steps 0" ab/conv_old.so $NEW 3 &&
grep -o '"ms_per_step": [0-9.]*\|== .*' gpurun_out/r06z/n.txt &&
for L in ab/conv_old.so $NEW ab/conv_old.so $NEW; do
  ADR_LIB=$L timeout -k 10 300 python -u bench.py --scale l --img 1280 --bs 16 --steps 8 --warmup 3 --roofline-steps 0 --stage-check 0 --no-cpu-baseline --infer-steps 0 --augment-bench 0 > gpurun_out/r06z/l.log 2>&1 || exit 1
  echo "$L $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r06z/l.log)"
done
