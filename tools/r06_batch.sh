#!/bin/bash
# Records placements on an 8 GiB file by batch size and ring depth (fill / drain of the host
# hashing against its steady rate).
set -o pipefail
OUT=gpurun_out/r06batch; rm -rf $OUT; mkdir -p $OUT
for b in 16 32 64; do
  for d in 0 8; do
    timeout -k 10 100 python -u tools/records_bench.py --gib 8 --modes host,hybrid --reps 3 --batch $b --depth $d > $OUT/rb_b${b}_d${d}.jsonl 2>&1 || exit 1
  done
done
timeout -k 10 100 python -u tools/records_bench.py --gib 8 --modes hybrid --reps 2 --batch 16 --stream 4 > $OUT/rb_b16_stream.jsonl 2>&1 || exit 1
timeout -k 10 100 python -u tools/records_bench.py --gib 8 --modes hybrid --reps 2 --batch 32 --stream 4 > $OUT/rb_b32_stream.jsonl 2>&1 || exit 1
grep -h best_GBps $OUT/*.jsonl | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['mode'], d['batch_segments'], d['depth'], d['window'], d['best_GBps'], d['seconds'], d['cpu_seconds'])"
grep -h records_stream $OUT/*.jsonl
