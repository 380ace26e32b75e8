#!/bin/bash
# GPU-only record hashing with and without the batch ramp, with the pipeline trace.
set -o pipefail
OUT=gpurun_out/r06gpumode; rm -rf $OUT; mkdir -p $OUT
for v in on off; do
  if [ $v = off ]; then export CEC_PIPELINE_NO_RAMP=1; else unset CEC_PIPELINE_NO_RAMP; fi
  CEC_PIPELINE_TRACE=1 timeout -k 10 150 python -u tools/records_bench.py --gib 8 --modes gpu --reps 2 > $OUT/rb_$v.jsonl 2>&1 || exit 1
  echo "== $v"; grep -v "destroy\|amdgpu" $OUT/rb_$v.jsonl | cut -c1-330
done
