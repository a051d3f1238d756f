# GPU suite on the tree, then same-box A/Bs: (1) nc_collapse's flat per-output kernel (in-tree) vs HEAD's eltwise
# (ab/ncc_old.so); (2) MLCA weight-gradient rows reduced at the flush (ADR_DEFER_MLCA=1) vs in the MLCA backward
mkdir -p gpurun_out/r06q
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06q/tests.log 2>&1 || { tail -30 gpurun_out/r06q/tests.log; exit 1; }
CMD="python bench.py --no-cpu-baseline --steps 40 --warmup 10 --infer-steps 0 --roofline-steps 0 --stage-check 0 --augment-bench 0 --lscale-steps 0 | grep -o '\"ms_per_step\": [0-9.]*'"
bash scripts/ab_lib.sh gpurun_out/r06q/ab_ncc.txt "$CMD" yolo-ad-refine_amd/adrefine/lib/libadr_hip.so ab/ncc_old.so 3 || exit 1
bash scripts/ab_env3.sh r06q/mlca "ADR_DEFER_MLCA=1" "ADR_DEFER_MLCA=0" 3 > gpurun_out/r06q/ab_mlca.txt 2>&1
