#!/bin/bash
# Does the bench's stream source (pieces of one 8 GiB buffer) make the opt-in resume slow?
# records_bench with --pieces, resume on / off, alternating.
set -o pipefail
OUT=gpurun_out/r06respieces; rm -rf $OUT; mkdir -p $OUT
for rep in 1 2; do
  for v in on off; do
    if [ $v = on ]; then export CEC_PIPELINE_RESUME=1; else unset CEC_PIPELINE_RESUME; fi
    CEC_PIPELINE_TRACE=1 timeout -k 10 200 python -u tools/records_bench.py --gib 8 --modes hybrid --reps 1 --stream 4 --pieces > $OUT/rb_${v}_$rep.jsonl 2>&1 || exit 1
    echo "== $v $rep"; grep -h "records_stream" $OUT/rb_${v}_$rep.jsonl | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d.get('GBps'), d.get('cpu_seconds'), d.get('file_done_s'))"
    grep "cec_pipeline" $OUT/rb_${v}_$rep.jsonl | tail -1 | cut -c1-170
  done
done
