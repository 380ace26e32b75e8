#!/bin/bash
# hybrid pipeline (C driver, 62.5 GiB): HW queue count / parity-copy stream priority
set -o pipefail
OUT=gpurun_out/r06q; rm -rf $OUT; mkdir -p $OUT
gcc -O2 -pthread tests/native/pipeline_e2e.c -Iinclude -Lcess_amd -lcessec -Loracle/build -loracle \
  -Wl,-rpath,$PWD/cess_amd:$PWD/oracle/build -o $OUT/pipeline_e2e || exit 1
run() { echo "== $*" >> $OUT/e2e.log; env "$@" CEC_PIPELINE_TRACE=1 timeout -k 10 120 $OUT/pipeline_e2e 2 1 8388608 4000 64 3 3 0 64 97 0 >> $OUT/e2e.log 2>&1 || exit 1; }
run X=0
run GPU_MAX_HW_QUEUES=8
run CEC_PIPELINE_D2H_PRIO=1
run CEC_PIPELINE_D2H_PRIO=0
run GPU_MAX_HW_QUEUES=8 X=1
grep -v "^W2026\|^E2026" $OUT/e2e.log | cut -c1-330
