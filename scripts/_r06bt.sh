# l-scale per-conv-shape table (eager step, HIP events per launch), sorted by time above the attainable roofline
mkdir -p gpurun_out/r06bt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u scripts/conv_table.py --scale l --img 1280 --bs 16 --steps 1 --by-gap --top 60 > gpurun_out/r06bt/l_table.txt 2>&1 || { tail -20 gpurun_out/r06bt/l_table.txt; exit 1; }
head -45 gpurun_out/r06bt/l_table.txt
