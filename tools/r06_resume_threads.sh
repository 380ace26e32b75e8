#!/bin/bash
# Resume (with the tick slack) on / off when the host has fewer SHA threads than the CPU share:
# does moving the segment chain to the GPU pay once the host is the bottleneck? records_bench's
# four-file stream, pieces source, 16 / 8 / 6 host threads.
set -o pipefail
OUT=gpurun_out/r06resthr; rm -rf $OUT; mkdir -p $OUT
for th in 16 8 6; do
  for v in on off; do
    if [ $v = on ]; then export CEC_PIPELINE_RESUME=1; else unset CEC_PIPELINE_RESUME; fi
    timeout -k 10 200 python -u tools/records_bench.py --gib 8 --modes hybrid --reps 1 --stream 4 --pieces --threads $th > $OUT/rb_${v}_$th.jsonl 2>&1 || exit 1
    echo "== $v threads=$th"; grep -h "records_stream" $OUT/rb_${v}_$th.jsonl | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d.get('GBps'), d.get('cpu_seconds'), d.get('file_done_s'))"
  done
done
