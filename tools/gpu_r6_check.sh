#!/bin/bash
# Round 6 check of the committed tree: the GPU suite, smoke, the default line, and the rocprof
# kernel-trace summary of the default line (profiles/r06/).
set -u
TAG=${1:-r06_check}
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
step pytest_gpu 900 python -u -m pytest tests -m gpu --maxfail=5 -v --timeout 200 --timeout-method thread
step smoke 180 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python -u bench.py
step rocprof_bench 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- python3 -u bench.py
echo done
