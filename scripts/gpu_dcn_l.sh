set -o pipefail
N=16 C=256 S=160 timeout -k 10 60 python scripts/dcn_bwd_micro.py 2>&1 | grep dcn_bwd || exit 1
N=16 C=128 S=160 timeout -k 10 60 python scripts/dcn_bwd_micro.py 2>&1 | grep dcn_bwd || exit 1
N=16 C=256 SIZES=160,80,40 timeout -k 10 200 python scripts/dcn_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
ADR_DCN_FUSED=0 N=16 C=256 SIZES=160,80,40 timeout -k 10 200 python scripts/dcn_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 200 python scripts/dcn_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
