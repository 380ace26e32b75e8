#!/bin/bash
# the C pipeline driven from C (tests/native/pipeline_e2e.c: 8-thread memcpy reader, no Python):
# 62.5 GiB source, host / hybrid placements at several ring depths, with the wait trace
set -o pipefail
rm -rf gpurun_out/r06e2e; mkdir -p gpurun_out/r06e2e
gcc -O2 -pthread tests/native/pipeline_e2e.c -Iinclude -Lcess_amd -lcessec -Loracle/build -loracle \
  -Wl,-rpath,$PWD/cess_amd:$PWD/oracle/build -o gpurun_out/r06e2e/pipeline_e2e || exit 1
for cfg in "0 3" "2 3" "3 3" "3 4" "3 6" "2 6"; do
  set -- $cfg
  CEC_PIPELINE_TRACE=1 timeout -k 10 120 gpurun_out/r06e2e/pipeline_e2e 2 1 8388608 4000 64 $2 $1 0 64 97 0 \
    >> gpurun_out/r06e2e/e2e.jsonl 2>> gpurun_out/r06e2e/trace.log || exit 1
done
cat gpurun_out/r06e2e/e2e.jsonl gpurun_out/r06e2e/trace.log | cut -c1-400
