# final tree: full GPU suite and smoke()
mkdir -p gpurun_out/r06cr
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash scripts/gpu_tests.sh r06cr tests/ || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu | tail -2
