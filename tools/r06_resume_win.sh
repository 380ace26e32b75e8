#!/bin/bash
# (Run while resume was the default and CEC_PIPELINE_NO_RESUME turned it off; it is now opt-in:
# set CEC_PIPELINE_RESUME=1 for the "on" legs to repeat it.)
# Hybrid (with resume) stream at hash windows 32 / 48 / 64, with the wait trace.
set -o pipefail
OUT=gpurun_out/r06reswin; rm -rf $OUT; mkdir -p $OUT
for rep in 1 2; do
  for w in 32 48 64; do
    CEC_PIPELINE_TRACE=1 timeout -k 10 150 python -u tools/records_bench.py --gib 1 --modes hybrid --reps 1 --stream 4 --window $w > $OUT/rb_w${w}_$rep.jsonl 2>&1 || exit 1
    echo "== window $w $rep"; grep -h "records_stream" $OUT/rb_w${w}_$rep.jsonl | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d.get('GBps'), d.get('cpu_seconds'), d.get('file_done_s'))"
    grep "cec_pipeline" $OUT/rb_w${w}_$rep.jsonl | tail -1 | cut -c1-150
  done
done
