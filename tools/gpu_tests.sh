#!/bin/bash
# GPU parity suite + smoke (+ optional extra steps), stopping at the first crash/abort/timeout.
# usage: tools/gpu_tests.sh <tag> [pytest -k expr]
set -u
TAG=${1:-r02}; K=${2:-}
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
if [ -n "$K" ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K"
else
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
fi
step smoke 180 python -u -c "import __graft_entry__ as g; g.smoke()"
echo done
