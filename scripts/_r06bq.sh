# TSSA token loops with four 16-byte loads in flight per thread at 256 threads: bitwise vs the HEAD kernels,
# packed-head / block tests, same-box bench A/B (n-scale and the l-scale object) against the HEAD library
mkdir -p gpurun_out/r06bq
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u scripts/tssa_ab.py ab/tssa_head.so 2>&1 | grep -v amdgpu
timeout -k 10 300 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_packed_head.py tests/test_gpu_blocks.py 2>&1 | tail -1
bash scripts/ab_lib.sh gpurun_out/r06bq/n.txt "python bench.py --no-cpu-baseline --steps 40 --infer-steps 0 --roofline-steps 0 --stage-check 0 --augment-bench 0 --lscale-steps 0" ab/tssa_head.so yolo-ad-refine_amd/adrefine/lib/libadr_hip.so 2 && grep -o '"ms_per_step": [0-9.]*\|== .*' gpurun_out/r06bq/n.txt
