#!/bin/bash
# Kernel stats of the GPU-only record placement, batch ramp on / off.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06gpuprof; rm -rf $OUT; mkdir -p $OUT
for v in on off; do
  if [ $v = off ]; then export CEC_PIPELINE_NO_RAMP=1; else unset CEC_PIPELINE_NO_RAMP; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v -o rb -- python3 -u tools/records_bench.py --gib 8 --modes gpu --reps 1 > $OUT/rb_$v.log 2>&1 || exit 1
  echo "== $v"; grep best_GBps $OUT/rb_$v.log | cut -c1-200
  f=$(find $OUT/$v -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 "$f" | head -8
done
