# same-box A/B: streaming (non-temporal) loads in the elementwise / BN-act kernels (in-tree) vs plain loads (ab/nt0.so)
mkdir -p gpurun_out/r06p
CMD="python bench.py --no-cpu-baseline --steps 40 --warmup 10 --infer-steps 0 --roofline-steps 0 --stage-check 0 --augment-bench 0 --lscale-steps 0 | grep -o '\"ms_per_step\": [0-9.]*'"
bash scripts/ab_lib.sh gpurun_out/r06p/ab.txt "$CMD" yolo-ad-refine_amd/adrefine/lib/libadr_hip.so ab/nt0.so 3
