# TSSA at 512 / 1024 threads (with the four-token load pipelining): arena drift of the packed-head test, then a
# same-box n-scale bench A/B against the in-tree 256-thread build
mkdir -p gpurun_out/r06bv
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for L in ab/tssa512.so ab/tssa1024.so; do
  echo "$L: $(ADR_LIB=$L timeout -k 10 200 python -u scripts/packed_arena_diff.py 2>&1 | grep 'arena rel')"
done
bash scripts/ab_lib.sh gpurun_out/r06bv/n.txt "python bench.py --no-cpu-baseline --steps 40 --infer-steps 0 --roofline-steps 0 --stage-check 0 --augment-bench 0 --lscale-steps 0" yolo-ad-refine_amd/adrefine/lib/libadr_hip.so ab/tssa512.so 2 && grep -o '"ms_per_step": [0-9.]*\|== .*' gpurun_out/r06bv/n.txt
