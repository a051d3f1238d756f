# stem: forward probes (no stores / no image loads), parity-split wgrad A/B + tests, SQ + TCC PMC of the forward
mkdir -p gpurun_out/r06be
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for P in 0 1 2 3; do
  ADR_STEM_PROBE=$P timeout -k 10 120 python -u scripts/stem_micro.py 64 640 16 20 > gpurun_out/r06be/p$P.txt 2>&1 || { tail -20 gpurun_out/r06be/p$P.txt; exit 1; }
  echo "probe $P: $(grep '\[1\] stem fwd' gpurun_out/r06be/p$P.txt)"
done
grep -v amdgpu gpurun_out/r06be/p0.txt
timeout -k 10 120 python -u scripts/stem_micro.py 2 320 32 5 | grep -v amdgpu
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu tests/test_gpu_conv.py -k stem tests/test_gpu_input.py > gpurun_out/r06be/tests.log 2>&1 || { tail -30 gpurun_out/r06be/tests.log; exit 1; }
tail -1 gpurun_out/r06be/tests.log
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -d gpurun_out/r06be/pmc1 -o pmc -- python3 scripts/stem_micro.py 64 640 16 2 > gpurun_out/r06be/pmc1.log 2>&1 || { tail -20 gpurun_out/r06be/pmc1.log; exit 1; }

python3 scripts/pmc_db_summary.py stem gpurun_out/r06be/pmc1 gpurun_out/r06be/pmc2
