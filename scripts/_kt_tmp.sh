cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for L in gw cur; do
  ADR_LIB=ab/dcn_$L.so ADR_DCN_BWD_MODE=2 R=3 timeout -k 10 90 rocprofv3 --kernel-trace -d gpurun_out/r05y/$L -o kt --output-format csv -- python3 scripts/dcn_bwd_micro.py || exit 1
done
