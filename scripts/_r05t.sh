set -o pipefail
timeout -k 10 300 python -u -m pytest -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu -k "packed or head" tests > gpurun_out/r05t_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05t_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_quick_bench.sh "attn or attention or c2p or psa or yolo11 or edffn or blocks or grads"
STEPS=12 bash scripts/prof_cmd.sh qw bench.py --no-cpu-baseline --steps 10 --warmup 2 --infer-steps 0 --stage-check 0 --augment-bench 0 --roofline-steps 0 > gpurun_out/prof_qw_summary.txt 2>&1; python3 - <<'P'
import csv
for r in csv.DictReader(open('gpurun_out/prof_qw/run_kernel_stats.csv')):
    n=r['Name']
    if any(t in n for t in ("bcast","attn_dvec")): print(n[:60], r['Calls'], r['AverageNs'])
P
