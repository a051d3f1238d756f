# generic implicit-GEMM column tile capped at 64 (the 128-wide double-buffered tile runs 2 workgroups per CU)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash scripts/ab_sweep.sh r06cf 3 "ADR_CONV_BN_MAX=64" &&
bash scripts/ab_sweep_l.sh r06cf_l 2 "ADR_CONV_BN_MAX=64"
