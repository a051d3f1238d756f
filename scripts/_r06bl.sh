mkdir -p gpurun_out/r06bl
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u scripts/tssa_ab.py 2>&1 | grep -v amdgpu
