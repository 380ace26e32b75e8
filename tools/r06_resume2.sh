#!/bin/bash
# (Run while resume was the default and CEC_PIPELINE_NO_RESUME turned it off; it is now opt-in:
# set CEC_PIPELINE_RESUME=1 for the "on" legs to repeat it.)
# Hybrid resume A/B, stream only (4 x 1000-segment files), three alternating pairs.
set -o pipefail
OUT=gpurun_out/r06resume2; rm -rf $OUT; mkdir -p $OUT
for rep in 1 2 3; do
  for v in on off; do
    if [ $v = off ]; then export CEC_PIPELINE_NO_RESUME=1; else unset CEC_PIPELINE_NO_RESUME; fi
    CEC_PIPELINE_TRACE=1 timeout -k 10 150 python -u tools/records_bench.py --gib 1 --modes hybrid --reps 1 --stream 4 > $OUT/rb_${v}_$rep.jsonl 2>&1 || exit 1
    echo "== $v $rep"; grep -h "records_stream" $OUT/rb_${v}_$rep.jsonl | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d.get('GBps'), d.get('cpu_seconds'), d.get('file_done_s'))"
    grep "cec_pipeline" $OUT/rb_${v}_$rep.jsonl | tail -1 | cut -c1-170
  done
done
