#!/bin/bash
# Kernel + memory-copy timeline of the C pipeline (64 GiB RS(2,1) file, GPU hashes, window 32).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/trace_e2e; mkdir -p $O
gcc -O2 -pthread tests/native/pipeline_e2e.c -Iinclude -Lcess_amd -lcessec -Loracle/build -loracle \
  -Wl,-rpath,$PWD/cess_amd:$PWD/oracle/build -o /tmp/pe2e || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O -o run -- \
  /tmp/pe2e 2 1 8388608 2048 64 3 1 32 64 1073741824 > $O/run.out 2>&1
rc=$?; tail -2 $O/run.out; exit $rc
