cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash scripts/ab_sweep_l.sh r06ce 2 "ADR_NC_ROWS=4096" "ADR_WG_MIN_KSTEPS=24" "ADR_WG_MIN_KSTEPS=8" "ADR_BN_XF_MAX_REUSE=250"
