# 3x3 halo-tile XF declined by default: XF / BSTAT / net / grads tests, then the full suite and the measurement set
mkdir -p gpurun_out/r06cj
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash scripts/gpu_tests.sh r06cj tests/ || exit 1
bash scripts/profile_r06.sh r06cj
