#!/bin/bash
# Records stream (4 x 1000-segment files): GPU-only and hybrid placements at hash windows 32 / 64,
# with the pipeline's wait trace.
set -o pipefail
OUT=gpurun_out/r06gpustream; rm -rf $OUT; mkdir -p $OUT
for w in 32 64; do
  CEC_PIPELINE_TRACE=1 timeout -k 10 200 python -u tools/records_bench.py --gib 1 --modes gpu,hybrid --reps 1 --stream 4 --window $w > $OUT/rb_w$w.jsonl 2>&1 || exit 1
  echo "== window $w"; grep -v "destroy\|amdgpu" $OUT/rb_w$w.jsonl | grep -v '"seconds": \[' | cut -c1-300
done
