# WGRAD DB with straight-line VMEM (vmcnt-counted stores): bitwise check, micro, l-scale and n-scale A/B
mkdir -p gpurun_out/r06w
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ADR_WG_DB=0 timeout -k 10 120 python3 scripts/wgrad_db_check.py > gpurun_out/r06w/db0.txt 2>&1 &&
ADR_WG_DB=1 timeout -k 10 120 python3 scripts/wgrad_db_check.py > gpurun_out/r06w/db1.txt 2>&1 &&
tail -1 gpurun_out/r06w/db0.txt && tail -1 gpurun_out/r06w/db1.txt &&
for e in 0 1; do for sh in "16 160 160 512 512 1 1 1" "16 160 160 256 256 3 3 2" "16 80 80 256 256 1 1 1"; do
  ADR_WG_DB=$e timeout -k 10 60 python3 scripts/conv_micro.py wgrad $sh 20 >> gpurun_out/r06w/micro.txt 2>&1 || exit 1
done; done && grep -v amdgpu.ids gpurun_out/r06w/micro.txt &&
bash scripts/l1280_ab.sh r06w/l "ADR_WG_DB=0" "ADR_WG_DB=1" "ADR_WG_DB=0" "ADR_WG_DB=1" &&
bash scripts/ab_env3.sh r06w/n "ADR_WG_DB=0" "ADR_WG_DB=1" 2
