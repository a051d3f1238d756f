set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/l1280p
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/l1280p/prof -o run -- python3 bench.py --scale l --img 1280 --bs 16 --steps 3 --warmup 2 --roofline-steps 0 --stage-check 0 > gpurun_out/l1280p/prof.log 2>&1 || { tail gpurun_out/l1280p/prof.log; exit 1; }
f=$(find gpurun_out/l1280p/prof -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/l1280p/kernel_stats.csv
python3 scripts/kernel_breakdown.py gpurun_out/l1280p/kernel_stats.csv
python3 scripts/kstat_summary.py gpurun_out/l1280p/kernel_stats.csv 6 25
