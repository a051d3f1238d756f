# l-scale (configs[4]) replayed-step kernel breakdown: rocprofv3 kernel trace of bench.py --scale l --img 1280 --bs 16
mkdir -p gpurun_out/r06cm
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06cm/prof -o run -- python3 bench.py --scale l --img 1280 --bs 16 --steps 6 --warmup 3 --roofline-steps 0 --stage-check 0 --augment-bench 0 > gpurun_out/r06cm/prof.log 2>&1 || { tail -20 gpurun_out/r06cm/prof.log; exit 1; }
TRACE=$(find gpurun_out/r06cm/prof -name "*kernel_trace.csv" | head -1)
python3 scripts/replay_breakdown.py $TRACE --steps 4 --top 60 > gpurun_out/r06cm/replay.md 2>&1
rm -f $TRACE
