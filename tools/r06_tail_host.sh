#!/bin/bash
# The tail rule with the host's backlog (CEC_PIPELINE_TAIL_HOST=1) against the transfer-only rule:
# the pipeline tests with it on, then records_bench's hybrid lone file (8 and 16 GiB, five runs
# each) on / off alternating twice, and the four-file stream once each.
set -o pipefail
OUT=gpurun_out/r06tailhost; rm -rf $OUT; mkdir -p $OUT
CEC_PIPELINE_TAIL_HOST=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_pipeline.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
run() {  # name gib on|off [stream]
  if [ $3 = on ]; then export CEC_PIPELINE_TAIL_HOST=1; else unset CEC_PIPELINE_TAIL_HOST; fi
  CEC_PIPELINE_TRACE=1 timeout -k 10 240 python -u tools/records_bench.py --gib $2 --modes hybrid --reps 5 ${4:+--stream 4 --pieces} > $OUT/rb_$1.jsonl 2>&1 || exit 1
  echo "== $1"; grep -h '"mode": "hybrid"' $OUT/rb_$1.jsonl | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l)
    if 'seconds' in d and isinstance(d['seconds'], list): print(sorted(d['seconds']), d['cpu_seconds'])
    elif 'GBps' in d: print('stream', d.get('GBps'), d.get('cpu_seconds'))"
}
for rep in 1 2; do
  for v in on off; do
    run l8_${v}_$rep 8 $v
    run l16_${v}_$rep 16 $v
  done
done
run s_on 8 on 1
run s_off 8 off 1
# The variant (pipeline.cpp, CEC_PIPELINE_TAIL_HOST) was slower and was reverted:
# profiles/r06/tail_host_ab/, DESIGN.md §7.
