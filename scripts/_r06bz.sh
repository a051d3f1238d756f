mkdir -p gpurun_out/r06bz
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for L in ab/pre_loss.so yolo-ad-refine_amd/adrefine/lib/libadr_hip.so ab/pre_loss.so yolo-ad-refine_amd/adrefine/lib/libadr_hip.so; do
  echo "== $L"; ADR_LIB=$L timeout -k 10 120 python -u scripts/loss_micro.py 2>&1 | grep -v amdgpu | tail -4
done
