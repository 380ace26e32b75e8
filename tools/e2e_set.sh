#!/bin/bash
# End-to-end (host memory -> GPU -> host) rates of the C pipeline, PCIe-inclusive.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-e2e}; mkdir -p $O
gcc -O2 -pthread tests/native/pipeline_e2e.c -Iinclude -Lcess_amd -lcessec -Loracle/build -loracle \
  -Wl,-rpath,$PWD/cess_amd:$PWD/oracle/build -o /tmp/pe2e || exit 1
for args in "2 1 8388608 1024 64 3 0 16 64 1073741824" "2 1 8388608 4096 64 3 0 16 64 1073741824" \
            "2 1 8388608 1024 64 3 1 32 64 1073741824" "2 1 8388608 4096 64 3 1 32 64 1073741824" \
            "2 1 8388608 256 64 3 1 16 64 1073741824" "32 32 524288 1024 64 3 1 32 64 1073741824"; do
  timeout -k 10 300 /tmp/pe2e $args >> $O/e2e.jsonl || exit 1
done
cat $O/e2e.jsonl
