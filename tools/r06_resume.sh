#!/bin/bash
# (Run while resume was the default and CEC_PIPELINE_NO_RESUME turned it off; it is now opt-in:
# set CEC_PIPELINE_RESUME=1 for the "on" legs to repeat it.)
# Hybrid resume (fragment 0 on the host, the segment chain continued on the GPU) against
# CEC_PIPELINE_NO_RESUME=1: pipeline tests first, then the records placements, alternating.
set -o pipefail
OUT=gpurun_out/r06resume; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_pipeline.py tests/test_gpu_parity.py -k "pipeline or records or sharded or segment_list" \
  > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for rep in 1 2; do
  for v in on off; do
    if [ $v = off ]; then export CEC_PIPELINE_NO_RESUME=1; else unset CEC_PIPELINE_NO_RESUME; fi
    CEC_PIPELINE_TRACE=1 timeout -k 10 150 python -u tools/records_bench.py --gib 8 --modes hybrid --reps 3 --stream 4 > $OUT/rb_${v}_$rep.jsonl 2>&1 || exit 1
    echo "== $v $rep"; grep -h "best_GBps\|records_stream" $OUT/rb_${v}_$rep.jsonl | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['mode'], d.get('best_GBps'), d.get('seconds'), d.get('GBps'), d.get('cpu_seconds'), d.get('file_done_s'))"
    grep "cec_pipeline" $OUT/rb_${v}_$rep.jsonl | tail -1 | cut -c1-200
  done
done
