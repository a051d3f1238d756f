# stem forward: 64-pixel fast path of the MFMA steps; micro, stem / input / lscale tests, same-box bench A/B
mkdir -p gpurun_out/r06br
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u scripts/stem_micro.py 64 640 16 20 2>&1 | grep -v amdgpu
timeout -k 10 120 python -u scripts/stem_micro.py 16 1280 64 10 2>&1 | grep -v amdgpu | grep fwd
timeout -k 10 300 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_conv.py tests/test_gpu_input.py tests/test_gpu_net.py 2>&1 | tail -1
bash scripts/ab_lib.sh gpurun_out/r06br/n.txt "python bench.py --no-cpu-baseline --steps 40 --infer-steps 0 --roofline-steps 0 --stage-check 0 --augment-bench 0 --lscale-steps 0" ab/pre_fast.so yolo-ad-refine_amd/adrefine/lib/libadr_hip.so 2 && grep -o '"ms_per_step": [0-9.]*\|== .*' gpurun_out/r06br/n.txt
