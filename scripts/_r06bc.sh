# stem forward on quad images: micro A/B (n-scale, l-scale, ragged width), stem / input tests
mkdir -p gpurun_out/r06bc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u scripts/stem_micro.py 64 640 16 20 > gpurun_out/r06bc/micro.txt 2>&1 || { tail -20 gpurun_out/r06bc/micro.txt; exit 1; }
timeout -k 10 120 python -u scripts/stem_micro.py 16 1280 64 20 >> gpurun_out/r06bc/micro.txt 2>&1 || { tail -20 gpurun_out/r06bc/micro.txt; exit 1; }
timeout -k 10 120 python -u scripts/stem_micro.py 2 1000 32 5 >> gpurun_out/r06bc/micro.txt 2>&1 || { tail -20 gpurun_out/r06bc/micro.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r06bc/micro.txt
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu tests/test_gpu_conv.py -k stem tests/test_gpu_input.py > gpurun_out/r06bc/tests.log 2>&1 || { tail -30 gpurun_out/r06bc/tests.log; exit 1; }
tail -2 gpurun_out/r06bc/tests.log
