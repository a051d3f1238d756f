cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/pmc_conv; mkdir -p $OUT
timeout -k 10 60 python scripts/conv_micro.py fwd2 64 40 40 128 128 3 3 1 > $OUT/time.txt 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES --output-format csv -d $OUT/p1 -o run -- python scripts/conv_micro.py fwd2 64 40 40 128 128 3 3 1 5 > $OUT/p1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR --output-format csv -d $OUT/p2 -o run -- python scripts/conv_micro.py fwd2 64 40 40 128 128 3 3 1 5 > $OUT/p2.log 2>&1
echo rc=$?
