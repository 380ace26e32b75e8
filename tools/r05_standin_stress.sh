#!/bin/bash
# round 5: longer plans through the C-ABI degraded read at world 8 / 3 / 2 over the RCCL stand-in
# (many rounds back to back: staging reuse across rounds, group cuts), every fragment vs the oracle
set -o pipefail
o=gpurun_out/r05/standin_stress
mkdir -p $o
R=${GRAFT_REPO_ROOT:-$PWD}
g++ -std=c++17 -O2 -shared -fPIC -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include tests/native/rccl_standin.cpp \
  -L/opt/rocm/lib -lamdhip64 -Wl,-soname,librccl.so.1 -o $o/librccl.so.1 || exit 1
make -s -C oracle || exit 1
gcc -O2 -D__HIP_PLATFORM_AMD__ tests/native/dist_world_n.c -Iinclude -I/opt/rocm/include -Lcess_amd -lcessec \
  -Loracle/build -loracle -L/opt/rocm/lib -lamdhip64 -pthread \
  -Wl,-rpath,$R/cess_amd:$R/oracle/build:/opt/rocm/lib -o $o/dist_world_n || exit 1
run() {
  echo "== $*"
  LD_LIBRARY_PATH=$o:$LD_LIBRARY_PATH timeout -k 10 300 $o/dist_world_n "$@" || exit 1
}
run 8 2 1 4096 65536 0 -1
run 8 32 32 1100 4096 2 -1
run 3 32 32 1100 4096 1 -1 200
run 2 10 4 2000 8192 2 -1 7
run 8 4 2 3000 4096 1 -1
