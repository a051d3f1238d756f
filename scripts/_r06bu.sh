# smoke() as the driver runs it, on the final tree
mkdir -p gpurun_out/r06bu
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06bu/smoke.log 2>&1; echo "smoke rc=$?"; tail -5 gpurun_out/r06bu/smoke.log
