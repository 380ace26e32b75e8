#!/bin/bash
# Kernel timeline of the hybrid stream (with resume): tick, encode and copy kernels per batch.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06hprof; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT -o rb -- python3 -u tools/records_bench.py --gib 1 --modes hybrid --reps 1 --stream 2 > $OUT/rb.log 2>&1 || exit 1
grep records_stream $OUT/rb.log | cut -c1-200
find $OUT -name "*kernel_trace.csv" | head -1
