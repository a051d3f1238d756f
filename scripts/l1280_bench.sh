set -o pipefail
mkdir -p gpurun_out/l1280
timeout -k 10 600 python -u bench.py --scale l --img 1280 --bs 16 --steps 5 --warmup 2 --roofline-steps 1 > gpurun_out/l1280/bench.log 2>&1; rc=$?
tail -c 3000 gpurun_out/l1280/bench.log; exit $rc
