# configs[4] on one GPU: l-scale 1280^2 bs16 train step, bf16 and with the fp8 forward-conv engine
set -o pipefail
mkdir -p gpurun_out/l1280
timeout -k 10 500 python -u bench.py --scale l --img 1280 --bs 16 --steps 5 --warmup 2 --roofline-steps 1 > gpurun_out/l1280/bf16.log 2>&1 || { tail -5 gpurun_out/l1280/bf16.log; exit 1; }
timeout -k 10 500 python -u bench.py --scale l --img 1280 --bs 16 --steps 5 --warmup 2 --roofline-steps 1 --conv-fp8 > gpurun_out/l1280/fp8.log 2>&1 || { tail -5 gpurun_out/l1280/fp8.log; exit 1; }
for f in bf16 fp8; do grep -o '"value": [0-9.]*, "unit": "images/s", "n_gpus": 1, "steps": 5, "warmup": 2, "ms_per_step": [0-9.]*' gpurun_out/l1280/$f.log; done
