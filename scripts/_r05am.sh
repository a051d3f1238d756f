set -o pipefail
bash scripts/ab_lib.sh gpurun_out/r05am_dcn.txt "python scripts/dcn_bwd_micro.py && ADR_DCN_BWD_MODE=1 python scripts/dcn_bwd_micro.py" ab/base.so ab/gbase.so 2 || exit 1
timeout -k 10 700 python -u -m pytest -x -q -s --timeout 600 --timeout-method thread tests/test_gpu_bf16_train.py -k amp > gpurun_out/r05al.txt 2>&1
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 240 --timeout-method thread tests/test_gpu_grads.py -k every > gpurun_out/r05an.txt 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --infer-steps 0 --stage-check 0 --augment-bench 0 > gpurun_out/r05ao_bench.log 2>&1
