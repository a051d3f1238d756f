# the 3x3 halo-tile XF data gradient off (ADR_XF_CONV3=0) vs on: n-scale 4 runs each, l-scale 2 each
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash scripts/ab_sweep.sh r06ci 4 "ADR_XF_CONV3=0" "ADR_GN_FUSED_MAXHW=100" &&
bash scripts/ab_sweep_l.sh r06ci_l 2 "ADR_XF_CONV3=0"
