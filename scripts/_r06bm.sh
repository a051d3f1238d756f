mkdir -p gpurun_out/r06bm
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u scripts/packed_arena_diff.py --all > gpurun_out/r06bm/new.txt 2>&1
ADR_LIB=ab/tssa_old.so timeout -k 10 200 python -u scripts/packed_arena_diff.py --all > gpurun_out/r06bm/old.txt 2>&1
