#!/bin/bash
# Round 4, session b: the GPU suite, the destroy-under-load report (codec alone, then a dist handle
# and its codec), smoke, the default line, and the rocprof kernel summary of the default command.
set -u
TAG=${1:-r04_b}
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
step pytest_gpu 600 python -u -m pytest tests -m gpu --maxfail=5 -v --timeout 120 --timeout-method thread
step destroy_report 120 python -u -m pytest tests/test_gpu_multi.py -m gpu -s -q -k c_dist_from_c
step smoke 180 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python -u bench.py
step prof_default 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_default" -o run -- \
  python -u bench.py
find "$OUT" -name "*kernel_stats.csv" | while read f; do cp "$f" "$OUT/$(basename $(dirname $f))_kernel_stats.csv"; done
echo done
