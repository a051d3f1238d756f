set -o pipefail
OUT=gpurun_out/d1; mkdir -p $OUT
timeout -k 10 300 python scripts/conv_table.py > $OUT/conv_table.txt 2>&1 && \
timeout -k 10 300 python scripts/ew_sites.py > $OUT/ew_sites.txt 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 30 --warmup 2 --no-cpu-baseline --infer-steps 0 --roofline-steps 0 > $OUT/prof.log 2>&1
echo rc=$?
