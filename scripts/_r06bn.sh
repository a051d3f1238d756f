mkdir -p gpurun_out/r06bn
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u scripts/packed_arena_diff.py 2>&1 | grep -v amdgpu | head -4
timeout -k 10 300 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_packed_head.py tests/test_gpu_blocks.py 2>&1 | tail -2
