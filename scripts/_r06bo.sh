# parity-split stem weight gradient at the l-scale width (160-column segments, K 64): micro A/B + stem / input tests
mkdir -p gpurun_out/r06bo
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u scripts/stem_micro.py 64 640 16 20 2>&1 | grep -v amdgpu
timeout -k 10 120 python -u scripts/stem_micro.py 16 1280 64 10 2>&1 | grep -v amdgpu
timeout -k 10 120 python -u scripts/stem_micro.py 2 1280 32 5 2>&1 | grep -v amdgpu
timeout -k 10 300 python -u -m pytest -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu tests/test_gpu_conv.py -k stem tests/test_gpu_input.py tests/test_gpu_lscale.py 2>&1 | tail -2
