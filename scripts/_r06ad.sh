# finalize tests; DCN weight-gradient L2 behaviour at the n-scale levels (TCC hit / miss, FETCH / WRITE)
mkdir -p gpurun_out/r06ad
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu tests/test_gpu_finalize.py > gpurun_out/r06ad/fin_test.log 2>&1 || { tail -30 gpurun_out/r06ad/fin_test.log; exit 1; }; tail -2 gpurun_out/r06ad/fin_test.log &&
R=3 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum --output-format csv -d gpurun_out/r06ad/p1 -o run -- python3 scripts/dcn_wgrad_levels_micro.py > gpurun_out/r06ad/p1.log 2>&1 &&
R=3 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/r06ad/p2 -o run -- python3 scripts/dcn_wgrad_levels_micro.py > gpurun_out/r06ad/p2.log 2>&1 &&
R=3 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/r06ad/p3 -o run -- python3 scripts/dcn_wgrad_levels_micro.py > gpurun_out/r06ad/p3.log 2>&1
