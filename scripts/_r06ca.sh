# knob sweep on the final tree: statistics chunk rows, WGRAD split floor / partial budget, cls anchors per group
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash scripts/ab_sweep.sh r06ca 2 "ADR_NC_ROWS=128" "ADR_NC_ROWS=512" "ADR_WG_MIN_KSTEPS=8" "ADR_WG_MIN_KSTEPS=24" "ADR_WG_PART_MB=48" "ADR_CLS_APB=64"
