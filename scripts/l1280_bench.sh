# configs[4]: the l-scale 701 model at 1280^2 bs 16 on one GPU, bf16 and with the fp8 forward convs
set -o pipefail
mkdir -p gpurun_out/l1280
timeout -k 10 600 python -u bench.py --scale l --img 1280 --bs 16 --steps 10 --warmup 3 --roofline-steps 1 --stage-check 0 > gpurun_out/l1280/bench.log 2>&1 || { tail -20 gpurun_out/l1280/bench.log; exit 1; }
grep '^{' gpurun_out/l1280/bench.log | tail -1 > gpurun_out/l1280/bench.json
timeout -k 10 600 python -u bench.py --scale l --img 1280 --bs 16 --steps 10 --warmup 3 --roofline-steps 0 --stage-check 0 --conv-fp8 > gpurun_out/l1280/bench_fp8.log 2>&1 || { tail -20 gpurun_out/l1280/bench_fp8.log; exit 1; }
grep '^{' gpurun_out/l1280/bench_fp8.log | tail -1 > gpurun_out/l1280/bench_fp8.json
python -c "
import json
for f in ('bench', 'bench_fp8'):
    d = json.load(open('gpurun_out/l1280/%s.json' % f))
    r = d.get('roofline') or {}
    print(f, d['ms_per_step'], d['value'], d['dtype'], (r.get('network') or {}), d['peak_hbm_gib'])
"
