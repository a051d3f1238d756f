# A/B of loss_cls_grad_kernel's anchors per workgroup (ADR_CLS_APB)
set -o pipefail
OUT=gpurun_out/${1:-lab}; mkdir -p $OUT
for apb in 256 64 32 16; do
  echo -n "apb=$apb " >> $OUT/ab.txt
  ADR_CLS_APB=$apb timeout -k 10 120 python scripts/loss_micro.py 2>>$OUT/err.txt | tail -1 >> $OUT/ab.txt || exit 1
done
