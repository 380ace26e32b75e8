#!/bin/bash
set -o pipefail
OUT=gpurun_out/r06rb; rm -rf $OUT; mkdir -p $OUT
for cfg in "--depth 0" "--depth 0 --window 64" "--depth 5 --window 64"; do
  echo "== $cfg" >> $OUT/rb.jsonl
  timeout -k 10 200 python -u tools/records_bench.py --gib 8 --modes hybrid --tails=-1,0 --reps 3 --stream 4 $cfg >> $OUT/rb.jsonl 2>&1 || exit 1
done
grep -v "amdgpu\|destroy" $OUT/rb.jsonl
