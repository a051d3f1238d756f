# tiled weight pack (coalesced KRSC + CRSK stores): pack-cache test, l- and n-scale A/B against the HEAD build.
# The HEAD library lacks adr_pack_weight2_tiled, so the A leg runs the HEAD python too (git-free: a copy of the tree
# is not available on the box) -> compare steps with the NEW library only against the committed r06ag numbers
mkdir -p gpurun_out/r06ai
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_graph.py tests/test_gpu_packed_head.py tests/test_abi.py > gpurun_out/r06ai/tests.log 2>&1 || { tail -30 gpurun_out/r06ai/tests.log; exit 1; }; tail -1 gpurun_out/r06ai/tests.log &&
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --scale l --img 1280 --bs 16 --steps 8 --warmup 3 --roofline-steps 0 --stage-check 0 --no-cpu-baseline --infer-steps 0 --augment-bench 0 > gpurun_out/r06ai/l.log 2>&1 || exit 1
  echo "l $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r06ai/l.log)"
done &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06ai/prof -o run -- python3 bench.py --scale l --img 1280 --bs 16 --steps 4 --warmup 2 --roofline-steps 0 --stage-check 0 --no-cpu-baseline --infer-steps 0 --augment-bench 0 > gpurun_out/r06ai/prof.log 2>&1 &&
grep -h "pack_weight2" gpurun_out/r06ai/prof/*kernel_stats.csv | cut -c1-160; rm -f gpurun_out/r06ai/prof/*kernel_trace.csv
