# bisect the packed-head fp32 arena drift: TSSA kernels / DCN kernels before their round-6 rewrites, presum off
mkdir -p gpurun_out/r06bj
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="tests/test_gpu_packed_head.py::test_trainer_packed_matches_levels"
for E in "ADR_LIB=ab/tssa_old.so" "ADR_LIB=ab/dcn_old.so" "ADR_FIN_PRESUM=0" "ADR_GN_GATE=0"; do
  env $E timeout -k 10 300 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu "$T" > gpurun_out/r06bj/t.log 2>&1; echo "[$E] $(tail -1 gpurun_out/r06bj/t.log)"; grep -E "^E  .*Assert" gpurun_out/r06bj/t.log | head -2
done
