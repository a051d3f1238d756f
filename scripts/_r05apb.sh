# loss_cls_grad_kernel time vs anchors per workgroup (ADR_CLS_APB), kernel-trace stats of a short bench each
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for a in 16 32 64 128; do
  O=gpurun_out/r05apb/$a; mkdir -p $O
  ADR_CLS_APB=$a timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 bench.py --no-cpu-baseline --steps 4 --warmup 2 --infer-steps 0 --stage-check 0 --augment-bench 0 --roofline-steps 0 > $O/log.txt 2>&1 || exit 1
  python3 -c "
import csv,glob
f=glob.glob('$O/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'loss_cls_grad' in r['Name'] or 'tal_topk' in r['Name']: print($a, r['Name'][:40], r['Calls'], r['AverageNs'])"
done
