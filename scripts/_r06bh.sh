# packed-head fp32 arena test under both stem settings, then the whole GPU suite (no -x), then the bench A/B
mkdir -p gpurun_out/r06bh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for E in "ADR_STEM_FWD_Q=0 ADR_STEM_WG_Q=0" "ADR_STEM_FWD_Q=1"; do
  env $E timeout -k 10 300 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_packed_head.py > gpurun_out/r06bh/ph.log 2>&1; echo "[$E] $(tail -1 gpurun_out/r06bh/ph.log)"; grep -E "^E  .*Assert" gpurun_out/r06bh/ph.log | head -3
done
bash scripts/gpu_tests.sh r06bh tests/
bash scripts/ab_env2.sh r06bh/ab "ADR_STEM_FWD_Q=0 ADR_STEM_WG_Q=0" "ADR_STEM_FWD_Q=1" 3
