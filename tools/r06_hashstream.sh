#!/bin/bash
# Hash-queue stream placement A/B: ticks on the encode stream (0) or their own stream (1 normal,
# 2 high, 3 low priority), and the default against GPU_MAX_HW_QUEUES=8; GPU-only and hybrid
# placements on the 4-file stream and an 8 GiB file, with the wait trace. The
# CEC_PIPELINE_HASH_STREAM knob existed for this measurement only (profiles/r06/hash_stream_ab/):
# no variant beat the ticks on the encode stream, and it was removed.
set -o pipefail
OUT=gpurun_out/r06hs; rm -rf $OUT; mkdir -p $OUT
run() {  # tag, then env assignments
  local tag=$1; shift
  env "$@" CEC_PIPELINE_TRACE=1 timeout -k 10 200 python -u tools/records_bench.py --gib 8 --modes gpu,hybrid --reps 2 --stream 4 > $OUT/rb_$tag.jsonl 2>&1 || return 1
  echo "== $tag"; grep -h "best_GBps\|records_stream" $OUT/rb_$tag.jsonl | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['mode'], d.get('best_GBps'), d.get('seconds'), d.get('GBps'), d.get('file_done_s'))"
  grep "cec_pipeline" $OUT/rb_$tag.jsonl | sed -n '2p;6p' | cut -c1-140
}
run s0 CEC_PIPELINE_HASH_STREAM=0 || exit 1
run s1 CEC_PIPELINE_HASH_STREAM=1 || exit 1
run s2 CEC_PIPELINE_HASH_STREAM=2 || exit 1
run s3 CEC_PIPELINE_HASH_STREAM=3 || exit 1
run s0_q8 CEC_PIPELINE_HASH_STREAM=0 GPU_MAX_HW_QUEUES=8 || exit 1
run s1_q8 CEC_PIPELINE_HASH_STREAM=1 GPU_MAX_HW_QUEUES=8 || exit 1
