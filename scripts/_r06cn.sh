# the XF data gradient off entirely (ADR_BN_XF_BWD=0) vs the default: n-scale 4 runs, l-scale 3 runs each
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash scripts/ab_sweep.sh r06cn 4 "ADR_BN_XF_BWD=0" &&
bash scripts/ab_sweep_l.sh r06cn_l 3 "ADR_BN_XF_BWD=0"
