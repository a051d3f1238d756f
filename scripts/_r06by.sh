# classification-loss kernel with prefetched anchor metadata / logit rows: bitwise arena A/B (fp32), loss tests,
# and a same-box bench A/B against the previous build
mkdir -p gpurun_out/r06by
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ADR_LIB=ab/pre_loss.so timeout -k 10 200 python -u scripts/arena_digest.py gpurun_out/r06by/a.pt 2>&1 | grep -v amdgpu
timeout -k 10 200 python -u scripts/arena_digest.py gpurun_out/r06by/b.pt 2>&1 | grep -v amdgpu
python -u scripts/arena_digest.py --compare gpurun_out/r06by/a.pt gpurun_out/r06by/b.pt
timeout -k 10 300 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_loss.py tests/test_gpu_trainer.py tests/test_gpu_bf16.py 2>&1 | tail -1
bash scripts/ab_lib.sh gpurun_out/r06by/n.txt "python bench.py --no-cpu-baseline --steps 40 --infer-steps 0 --roofline-steps 0 --stage-check 0 --augment-bench 0 --lscale-steps 0" ab/pre_loss.so yolo-ad-refine_amd/adrefine/lib/libadr_hip.so 2 && grep -o '"ms_per_step": [0-9.]*\|== .*' gpurun_out/r06by/n.txt
