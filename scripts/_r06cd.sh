# second knob sweep on the final tree (NC_ROWS 1024 default): statistics min blocks, BN-act XF reuse thresholds
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash scripts/ab_sweep.sh r06cd 3 "ADR_NC_MIN_BLOCKS=256" "ADR_NC_MIN_BLOCKS=1024" "ADR_NC_ROWS=2048" "ADR_BN_XF_MAX_REUSE=250" "ADR_BN_XF_FWD_MAX_REUSE=300"
