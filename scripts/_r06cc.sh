# full GPU suite, then the round's measurement set (PMC calibration, traffic, replay table, default bench line)
mkdir -p gpurun_out/r06cc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash scripts/gpu_tests.sh r06cc tests/ || exit 1
bash scripts/profile_r06.sh r06cc
