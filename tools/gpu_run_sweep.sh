#!/bin/bash
# The decoder chooser on consecutive-erasure patterns (--erasure-run): each decoder forced, then
# the default, one process each (30 warm-up launches, 20 timed), at 12..32 erasures.
set -u
TAG=${1:-r04_runsweep}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
: > "$OUT/sweep.jsonl"
for e in 12 16 20 24 28 32; do
  for opt in "--fftdec-mode 1" "--fftdec-mode 2" "--fftdec-min 0" ""; do
    timeout -k 10 90 python -u bench.py --config 6 --erasures $e --erasure-run $opt --steps 20 \
      --no-cpu-baseline --no-extra >> "$OUT/sweep.jsonl" 2> "$OUT/err.log" || { echo "e$e '$opt' rc=$?"; tail -5 "$OUT/err.log"; exit 1; }
  done
  echo "e$e done"
done
