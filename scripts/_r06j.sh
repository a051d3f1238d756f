mkdir -p gpurun_out/r06j
for m in 0 1 2; do
  ADR_DCN_BWD_MODE=$m SPREAD=0.5 timeout -k 10 120 python scripts/dcn_bwd_micro.py >> gpurun_out/r06j/micro.txt 2>&1 || exit 1
done
for s in 40 20; do
  S=$s SPREAD=0.5 timeout -k 10 120 python scripts/dcn_bwd_micro.py >> gpurun_out/r06j/micro.txt 2>&1 || exit 1
done
