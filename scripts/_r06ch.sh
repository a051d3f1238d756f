# third n-scale knob sweep (switches tuned in earlier rounds, re-checked on the final tree)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash scripts/ab_sweep.sh r06ch 2 "ADR_DG2H=2" "ADR_DG2H=0" "ADR_GN_FUSED_MAXHW=1600" "ADR_GN_FUSED_MAXHW=100" "ADR_CONV3W=0" "ADR_XF_CONV3=0" "ADR_EDFFN_MFMA=0" "ADR_WG_DB=0"
