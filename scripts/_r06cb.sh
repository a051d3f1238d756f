cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash scripts/ab_sweep.sh r06cb 4 "ADR_NC_ROWS=512" "ADR_NC_ROWS=1024" "ADR_WG_MIN_KSTEPS=24" "ADR_NC_ROWS=512 ADR_WG_MIN_KSTEPS=24"
