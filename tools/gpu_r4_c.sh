#!/bin/bash
# Round 4, session c: the destroy report (codec, dist handle, bare RCCL teardown control), the
# multi-rank GPU tests, and the two-rank rehearsal of the multi-GPU line (ranks sharing GPU 0).
set -u
TAG=${1:-r04_c}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 tmo=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  if grep -q "illegal memory access\|Memory access fault\|HSA_STATUS_ERROR" "$OUT/$name.log"; then
    echo "stopping after $name: GPU fault"; exit 3; fi
  return 0
}
step destroy_report 120 python -u -m pytest tests/test_gpu_multi.py -m gpu -s -v -k c_dist_from_c
step multi 400 python -u -m pytest tests/test_gpu_multi.py -m gpu -v --timeout 200 --timeout-method thread
CESS_DIST_BACKEND=gloo CESS_DEVICE=0 step bench_gpus2_gloo 400 python -u bench.py --gpus 2 --steps 20
echo done
