mkdir -p gpurun_out/r06bi
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u scripts/packed_arena_diff.py 2>&1 | grep -v amdgpu
