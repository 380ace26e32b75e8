#!/bin/bash
# kernel / copy timeline of the hybrid pipeline (C driver, 62.5 GiB source)
set -o pipefail
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/r06e2eprof; rm -rf $OUT; mkdir -p $OUT
gcc -O2 -pthread tests/native/pipeline_e2e.c -Iinclude -Lcess_amd -lcessec -Loracle/build -loracle \
  -Wl,-rpath,$PWD/cess_amd:$PWD/oracle/build -o $OUT/pipeline_e2e || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/prof -o e2e -- \
  $OUT/pipeline_e2e 2 1 8388608 1000 64 3 3 0 64 97 0 > $OUT/run.log 2>&1 || { tail -5 $OUT/run.log; exit 1; }
cat $OUT/run.log | tail -2
find $OUT/prof -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-160
