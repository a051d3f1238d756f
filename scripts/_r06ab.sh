# two-level BN finalize: micro, tests, n-scale A/B (ADR_FIN_PRESUM=0 vs 1)
mkdir -p gpurun_out/r06ab
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 scripts/finalize_micro.py > gpurun_out/r06ab/micro.txt 2>&1 && grep -v amdgpu.ids gpurun_out/r06ab/micro.txt &&
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu tests/test_gpu_finalize.py tests/test_gpu_bstat.py tests/test_gpu_net.py > gpurun_out/r06ab/tests.log 2>&1 || { tail -30 gpurun_out/r06ab/tests.log; exit 1; }; tail -3 gpurun_out/r06ab/tests.log &&
bash scripts/ab_env3.sh r06ab/n "ADR_FIN_PRESUM=0" "ADR_FIN_PRESUM=1" 3
