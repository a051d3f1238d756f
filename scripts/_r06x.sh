# WGRAD partial budget at l-scale (split count of the long 1x1 / 3x3-s2 weight gradients)
mkdir -p gpurun_out/r06x
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for e in "ADR_WG_PART_MB=24" "ADR_WG_PART_MB=96"; do
  env $e timeout -k 10 60 python3 scripts/conv_micro.py wgrad 16 160 160 512 512 1 1 1 20 >> gpurun_out/r06x/micro.txt 2>&1 || exit 1
done && grep -v amdgpu.ids gpurun_out/r06x/micro.txt &&
bash scripts/l1280_ab.sh r06x/l "X=0" "ADR_WG_PART_MB=64" "ADR_WG_PART_MB=160" "X=0" "ADR_WG_PART_MB=64" "ADR_WG_PART_MB=160"
