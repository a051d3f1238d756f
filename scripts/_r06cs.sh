# final tree: the round's measurement set (PMC calibration, traffic, replay table, default bench line)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash scripts/profile_r06.sh r06cs
