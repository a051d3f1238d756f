# l-scale A/B: long 1x1 reductions on the 128-wide double-buffered conv tile (ADR_C1_DB_MINRED); WGRAD 1x1 PMC
mkdir -p gpurun_out/r06v
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash scripts/l1280_ab.sh r06v/l "ADR_C1_DB_MINRED=0" "ADR_C1_DB_MINRED=512" "ADR_C1_DB_MINRED=256" "ADR_C1_DB_MINRED=0" "ADR_C1_DB_MINRED=512" &&
for m in fwd2 dgrad2; do for e in 0 512; do
  ADR_C1_DB_MINRED=$e timeout -k 10 60 python3 scripts/conv_micro.py $m 16 160 160 512 512 1 1 1 20 >> gpurun_out/r06v/micro.txt 2>&1 || exit 1
  ADR_C1_DB_MINRED=$e timeout -k 10 60 python3 scripts/conv_micro.py $m 16 80 80 1024 512 1 1 1 20 >> gpurun_out/r06v/micro.txt 2>&1 || exit 1
done; done &&
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES --output-format csv -d gpurun_out/r06v/pmc1 -o run -- python3 scripts/conv_micro.py wgrad 16 160 160 512 512 1 1 1 5 > gpurun_out/r06v/pmc1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES --output-format csv -d gpurun_out/r06v/pmc2 -o run -- python3 scripts/conv_micro.py wgrad 16 160 160 256 256 3 3 2 5 > gpurun_out/r06v/pmc2.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum --output-format csv -d gpurun_out/r06v/pmc3 -o run -- python3 scripts/conv_micro.py wgrad 16 160 160 512 512 1 1 1 5 > gpurun_out/r06v/pmc3.log 2>&1
