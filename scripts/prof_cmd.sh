# rocprofv3 kernel-trace stats of a python command. usage: bash scripts/prof_cmd.sh <tag> <python args...>
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/prof_$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 "$@" > $OUT/log.txt 2>&1
rc=$?
f=$(find $OUT -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && python3 scripts/prof_summary.py "$f" ${STEPS:-1} 30
exit $rc
