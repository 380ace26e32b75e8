#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprof kernel stats. Stops at the first crash,
# abort or timeout (exit codes other than 0/1); ordinary test failures (1) do not stop it.
# usage: tools/gpu_check.sh <tag> [bench args...]
set -u
TAG=${1:-r01}; shift || true
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
step() {  # step <name> <timeout> cmd...
  local name=$1 tmo=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
step smoke 180 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python -u bench.py "$@"
cp "$OUT/bench.log" "$OUT/bench.json"
export TMPDIR=/tmp
step rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python -u bench.py --no-cpu-baseline --no-extra "$@"
find "$OUT/prof" -name "*kernel_stats*" -exec cp {} "$OUT/" \;
echo "done"
