# elementwise call sites of the n-scale step (where the 78 ew launches come from) + op table
mkdir -p gpurun_out/r06aa
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 scripts/ew_sites.py > gpurun_out/r06aa/ew_sites.txt 2>&1
