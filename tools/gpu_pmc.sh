#!/bin/bash
# PMC passes (one counter group per run, kernel-trace only) for a bench config.
# usage: tools/gpu_pmc.sh <tag> <config> <kernel-substring> <algorithmic-bytes-per-launch>
set -u
TAG=$1; CFG=$2; KERN=$3; ALGO=$4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$c" -o run -- \
    python -u bench.py --config "$CFG" --no-cpu-baseline --no-extra --steps 5 --warmup 1 \
    > "$OUT/pmc_$c.log" 2>&1 || { echo "pmc $c failed rc=$?"; tail -5 "$OUT/pmc_$c.log"; exit 1; }
done
F=$(find "$OUT/pmc_FETCH_SIZE" -name "*counter_collection.csv" | head -1)
W=$(find "$OUT/pmc_WRITE_SIZE" -name "*counter_collection.csv" | head -1)
python tools/pmc_traffic.py "$F" "$W" "$KERN" "$OUT/traffic_c$CFG.json" "$ALGO"
