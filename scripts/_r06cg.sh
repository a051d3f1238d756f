# generic conv column tile: 64 wide when the 128-wide grid is under 1024 workgroups (default now) vs never (128)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_conv.py tests/test_gpu_bnxf.py tests/test_gpu_bstat.py tests/test_gpu_dg2.py tests/test_gpu_net.py 2>&1 | tail -1
bash scripts/ab_sweep.sh r06cg 3 "ADR_CONV_BN_MAX=128" &&
bash scripts/ab_sweep_l.sh r06cg_l 2 "ADR_CONV_BN_MAX=128"
