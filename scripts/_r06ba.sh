# double-buffered narrow conv tile: micro (bitwise + times), then the per-shape conv table with it off / on
mkdir -p gpurun_out/r06ba
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u scripts/conv_db_micro.py 50 > gpurun_out/r06ba/micro.txt 2>&1 || { tail -20 gpurun_out/r06ba/micro.txt; exit 1; }
cat gpurun_out/r06ba/micro.txt
ADR_CONV_DB=0 timeout -k 10 300 python -u scripts/conv_table.py --steps 2 --by-gap > gpurun_out/r06ba/table0.txt 2>&1 || { tail -20 gpurun_out/r06ba/table0.txt; exit 1; }
ADR_CONV_DB=-1 timeout -k 10 300 python -u scripts/conv_table.py --steps 2 --by-gap > gpurun_out/r06ba/table1.txt 2>&1 || { tail -20 gpurun_out/r06ba/table1.txt; exit 1; }
head -3 gpurun_out/r06ba/table0.txt gpurun_out/r06ba/table1.txt
