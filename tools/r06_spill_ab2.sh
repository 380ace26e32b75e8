#!/bin/bash
# A/B of the tail spill on the hybrid records stream only (4 x 1000-segment files), alternating.
set -o pipefail
OUT=gpurun_out/r06spillab2; rm -rf $OUT; mkdir -p $OUT
for rep in 1 2 3; do
  for v in on off; do
    if [ $v = off ]; then export CEC_HOST_SHA_NO_SPILL=1; else unset CEC_HOST_SHA_NO_SPILL; fi
    timeout -k 10 150 python -u tools/records_bench.py --gib 1 --modes hybrid --reps 1 --stream 4 > $OUT/rb_${v}_$rep.jsonl 2>&1 || exit 1
    timeout -k 10 150 python -u tools/records_bench.py --gib 8 --modes host --reps 3 > $OUT/rbh_${v}_$rep.jsonl 2>&1 || exit 1
  done
done
unset CEC_HOST_SHA_NO_SPILL
for f in $OUT/*.jsonl; do echo "== $f"; grep -h "best_GBps\|records_stream" $f | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['mode'], d.get('best_GBps'), d.get('seconds'), d.get('GBps'), d.get('file_done_s'))"; done
