#!/bin/bash
# Tick producer with per-lane fast runs: hash-queue + pipeline GPU tests, then the GPU-only
# record placement with the batch ramp on / off (the case that mixed finished and running chains
# in one 64-chain group), with the pipeline trace.
set -o pipefail
OUT=gpurun_out/r06tickfix; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_hashq.py tests/test_gpu_pipeline.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for v in on off; do
  if [ $v = off ]; then export CEC_PIPELINE_NO_RAMP=1; else unset CEC_PIPELINE_NO_RAMP; fi
  CEC_PIPELINE_TRACE=1 timeout -k 10 150 python -u tools/records_bench.py --gib 8 --modes gpu,hybrid --reps 2 --stream 4 > $OUT/rb_$v.jsonl 2>&1 || exit 1
  echo "== $v"; grep -v "destroy\|amdgpu\|cec_pipeline" $OUT/rb_$v.jsonl | cut -c1-250
done
