# A/B of the concurrent head levels and the forward BN-act fusion under hipGraph replay, plus the HIP runtime's
# graph-execution knobs (host enqueue vs GPU time). usage: bash scripts/ab_levels.sh (GPU)
set -o pipefail
OUT=gpurun_out/ab_levels; mkdir -p $OUT
run() {  # label, env...
  local label=$1; shift
  echo -n "$label: "
  env "$@" timeout -k 10 240 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --infer-steps 0 --stage-check 0 \
      --augment-bench 0 --roofline-steps 1 > $OUT/$label.log 2>&1 || { echo FAIL; tail -5 $OUT/$label.log; return 1; }
  grep '^{' $OUT/$label.log | tail -1 | python -c "import json,sys;d=json.load(sys.stdin);print(d['ms_per_step'], 'host', d['host_enqueue_ms_per_step'], 'ev', d['ms_per_step_events'])"
}
run serial ADR_LEVEL_STREAMS=0 && \
run levels ADR_LEVEL_STREAMS=1 && \
run serial_noxf ADR_LEVEL_STREAMS=0 ADR_BN_XF_FWD=0 && \
run levels_q1 ADR_LEVEL_STREAMS=1 DEBUG_HIP_FORCE_GRAPH_QUEUES=1 && \
run levels_q4 ADR_LEVEL_STREAMS=1 DEBUG_HIP_FORCE_GRAPH_QUEUES=4 && \
run levels_b64 ADR_LEVEL_STREAMS=1 DEBUG_HIP_GRAPH_BATCH_SIZE=64 && \
run serial_nocap ADR_LEVEL_STREAMS=0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 && \
run levels_nocap ADR_LEVEL_STREAMS=1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 && \
run serial2 ADR_LEVEL_STREAMS=0 && \
run levels2 ADR_LEVEL_STREAMS=1
