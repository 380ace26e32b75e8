#!/bin/bash
# The exchange forms compared the way the line runs them: one form per process (30 warm-up
# launches, 50 timed), alternating processes on one box. -1 = the product (crossbar in the IFFT
# and derivative / the IFFT), 83 / 84 = DPP everywhere (tuning build).
set -u
TAG=${1:-r04_swz4}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
: > "$OUT/runs.jsonl"
for rep in 1 2 3; do
  for e in 32 16; do
    for v in -1 83; do
      timeout -k 10 120 python -u bench.py --config 6 --erasures $e --fftdec-mode 2 --variant $v \
        --steps 50 --warmup 30 --no-cpu-baseline --no-extra > "$OUT/one.log" 2>&1 || { tail -5 "$OUT/one.log"; exit 1; }
      grep '^{' "$OUT/one.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'e': $e, 'dec': 'd', 'variant': $v, 'ms': d['roofline']['launch_ms']}))" | tee -a "$OUT/runs.jsonl"
    done
  done
  for v in -1 84; do
    timeout -k 10 120 python -u bench.py --config 6 --erasures 8 --fftdec-mode 1 --variant $v \
      --steps 50 --warmup 30 --no-cpu-baseline --no-extra > "$OUT/one.log" 2>&1 || { tail -5 "$OUT/one.log"; exit 1; }
    grep '^{' "$OUT/one.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'e': 8, 'dec': 'm', 'variant': $v, 'ms': d['roofline']['launch_ms']}))" | tee -a "$OUT/runs.jsonl"
  done
done
