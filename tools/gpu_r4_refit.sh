#!/bin/bash
# Round 4: the GPU suite, smoke, the default line, the destroy-under-load report, and the warm
# sweep the decoder cost model is fitted on (config 6: random erasures per segment, each decoder
# forced: 1 syndrome rows, 2 formal derivative, and the run-time matrix kernels (fftdec-min 0)).
set -u
TAG=${1:-r04_refit}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
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
: > "$OUT/sweep.jsonl"
for e in 4 6 8 12 16 20 24 28 32; do
  for mode in 1 2; do
    timeout -k 10 90 python -u bench.py --config 6 --erasures $e --fftdec-mode $mode --steps 20 \
      --no-cpu-baseline --no-extra >> "$OUT/sweep.jsonl" 2> "$OUT/sweep_err.log" || { echo "sweep e$e m$mode rc=$?"; exit 1; }
  done
  timeout -k 10 90 python -u bench.py --config 6 --erasures $e --fftdec-min 0 --steps 20 \
    --no-cpu-baseline --no-extra >> "$OUT/sweep.jsonl" 2>> "$OUT/sweep_err.log" || { echo "sweep e$e rt rc=$?"; exit 1; }
  timeout -k 10 90 python -u bench.py --config 6 --erasures $e --steps 20 \
    --no-cpu-baseline --no-extra >> "$OUT/sweep.jsonl" 2>> "$OUT/sweep_err.log" || { echo "sweep e$e auto rc=$?"; exit 1; }
  echo "sweep e$e done"
done
echo done
