# WGRAD double-buffered 128x128 tile: bitwise check vs the single-stage kernel, then l-scale and n-scale A/B
mkdir -p gpurun_out/r06u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ADR_WG_DB=0 timeout -k 10 120 python3 scripts/wgrad_db_check.py > gpurun_out/r06u/db0.txt 2>&1 &&
ADR_WG_DB=1 timeout -k 10 120 python3 scripts/wgrad_db_check.py > gpurun_out/r06u/db1.txt 2>&1 &&
tail -1 gpurun_out/r06u/db0.txt && tail -1 gpurun_out/r06u/db1.txt &&
bash scripts/l1280_ab.sh r06u/l "ADR_WG_DB=0" "ADR_WG_DB=1" "ADR_WG_DB=0" "ADR_WG_DB=1" &&
bash scripts/ab_env3.sh r06u/n "ADR_WG_DB=0" "ADR_WG_DB=1" 2
