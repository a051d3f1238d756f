# DG2H (stride-2 halo-tile data gradient) vs the per-class implicit GEMM on the step's stride-2 shapes, then the
# same-box bench A/B. usage: bash scripts/gpu_dg2_ab.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-dg2}; mkdir -p $OUT
for shp in "64 320 320 16 32" "64 160 160 64 64" "64 80 80 128 128" "64 40 40 128 256" "64 40 40 128 128"; do
  for v in 1 0; do
    echo -n "DG2H=$v $shp: "; ADR_DG2H=$v timeout -k 10 60 python scripts/conv_micro.py dgrad2 $shp 3 3 2 50 2>&1 | tail -1 || exit 1
  done
done | tee $OUT/micro.txt
bash scripts/ab_env2.sh ${1:-dg2} "ADR_DG2H=1" "ADR_DG2H=0" 2
