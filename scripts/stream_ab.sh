# Whole-step A/B of the streaming-kernel grid caps: bench.py under several ADR_STREAM_BLOCKS / ADR_EW_BLOCKS
# settings on one box (0 = uncapped), alternating twice.
set -o pipefail
OUT=gpurun_out/${1:-sab}; mkdir -p $OUT
for rep in 1 2; do
  for cfg in "-1 -1" "0 0" "8192 8192" "4096 4096"; do
    set -- $cfg
    envs=""
    [ "$1" != "-1" ] && envs="ADR_STREAM_BLOCKS=$1 ADR_EW_BLOCKS=$2"
    echo -n "rep$rep cfg[$cfg] " >> $OUT/ab.txt
    env $envs timeout -k 10 300 python bench.py --no-cpu-baseline --infer-steps 0 --roofline-steps 1 --steps 20 \
      > $OUT/b.json 2>> $OUT/err.txt || exit 1
    python -c "import json; d=json.load(open('$OUT/b.json')); k=d['roofline']['kernels']; print(d['ms_per_step'], {n: v['avg_us'] for n, v in list(k.items())[:5]})" >> $OUT/ab.txt
  done
done
