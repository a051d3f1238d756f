mkdir -p gpurun_out/r06h
bash scripts/ab_env3.sh r06h/dcn "ADR_DCN_FAR_FRESH=0" "ADR_DCN_FAR_FRESH=1" 3 > gpurun_out/r06h/dcn.txt 2>&1 &&
bash scripts/ab_env3.sh r06h/gate "ADR_GN_GATE=1" "ADR_GN_GATE=0" 2 > gpurun_out/r06h/gate.txt 2>&1 &&
timeout -k 10 300 python scripts/torch_ops_stack.py > gpurun_out/r06h/ops.txt 2>&1
