# l-scale knob sweep (after the 3x3 XF decline)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash scripts/ab_sweep_l.sh r06ck 2 "ADR_BN_XF_FWD=0" "ADR_BN_BSTAT=0" "ADR_CONV3W=0" "ADR_DG2H=2" "ADR_WG_DB=0" "ADR_BN_XF_BWD=0"
