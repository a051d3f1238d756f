# stem kernels (quad forward with per-block statistics, parity-split weight gradient): micro, full GPU suite,
# same-box bench A/B against the row-gather kernels (ADR_STEM_FWD_Q=0 ADR_STEM_WG_Q=0)
mkdir -p gpurun_out/r06bg
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u scripts/stem_micro.py 64 640 16 20 2>&1 | grep -v amdgpu
bash scripts/gpu_tests.sh r06bg -x tests/ || exit 1
bash scripts/ab_env2.sh r06bg/ab "ADR_STEM_FWD_Q=0 ADR_STEM_WG_Q=0" "ADR_STEM_FWD_Q=1" 3
