#!/bin/bash
# Resume with the tick slack, on / off alternating: records_bench's four-file stream (pieces
# source, 16 threads) three times each, then the default bench line's host_e2e three times each.
set -o pipefail
OUT=gpurun_out/r06resab3; rm -rf $OUT; mkdir -p $OUT
setv() { if [ $1 = on ]; then export CEC_PIPELINE_RESUME=1; else unset CEC_PIPELINE_RESUME; fi; }
for rep in 1 2 3; do
  for v in on off; do
    setv $v
    timeout -k 10 200 python -u tools/records_bench.py --gib 8 --modes hybrid --reps 1 --stream 4 --pieces > $OUT/rb_${v}_$rep.jsonl 2>&1 || exit 1
    echo "== rb $v $rep"; grep -h "records_stream" $OUT/rb_${v}_$rep.jsonl | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d.get('GBps'), d.get('cpu_seconds'), d.get('file_done_s'))"
  done
done
for rep in 1 2 3; do
  for v in on off; do
    setv $v
    timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_${v}_$rep.log 2>&1 || exit 1
    echo "== bench $v $rep"; grep '^{' $OUT/bench_${v}_$rep.log | tail -1 | python -c "
import sys, json
d = json.loads(sys.stdin.read()); h = d['extra']['host_e2e']
print({k: (h[k].get('node_GBps'), h[k].get('cpu_s', h[k].get('cpu_s_runs'))) for k in ('segment_lists_hybrid', 'records_stream')})"
  done
done
