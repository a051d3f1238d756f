mkdir -p gpurun_out/r06bk
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ADR_LIB=ab/tssa_old.so timeout -k 10 200 python -u scripts/packed_arena_diff.py 2>&1 | grep -v amdgpu | head -8
timeout -k 10 200 python -u scripts/packed_arena_diff.py 2>&1 | grep -v amdgpu | head -3
