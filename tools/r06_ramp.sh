#!/bin/bash
# Batch ramp / tail split of the C pipeline: the pipeline tests, then an A/B against
# CEC_PIPELINE_NO_RAMP=1 (alternating) on the records placements of an 8 GiB file + the stream.
set -o pipefail
OUT=gpurun_out/r06ramp; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_pipeline.py tests/test_retrieve.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for rep in 1 2; do
  for v in on off; do
    if [ $v = off ]; then export CEC_PIPELINE_NO_RAMP=1; else unset CEC_PIPELINE_NO_RAMP; fi
    timeout -k 10 150 python -u tools/records_bench.py --gib 8 --modes none,host,hybrid --reps 3 --stream 4 > $OUT/rb_${v}_$rep.jsonl 2>&1 || exit 1
  done
done
unset CEC_PIPELINE_NO_RAMP
for f in $OUT/rb_*.jsonl; do echo "== $f"; grep -h "best_GBps\|records_stream" $f | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['mode'], d.get('best_GBps'), d.get('seconds'), d.get('GBps'), d.get('file_done_s'))"; done
