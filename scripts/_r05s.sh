set -o pipefail
bash scripts/gpu_quick_bench.sh "edffn or c2p or mona or tssa or blocks" && STEPS=12 bash scripts/prof_cmd.sh topk bench.py --no-cpu-baseline --steps 10 --warmup 2 --infer-steps 0 --stage-check 0 --augment-bench 0 --roofline-steps 0 > gpurun_out/prof_topk_summary.txt 2>&1; python3 - <<'P'
import csv
for r in csv.DictReader(open('gpurun_out/prof_topk/run_kernel_stats.csv')):
    n=r['Name']
    if any(t in n for t in ("edffn","dw_")): print(n[:60], r['Calls'], r['AverageNs'], r['MinNs'], r['MaxNs'])
P
