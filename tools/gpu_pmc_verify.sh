#!/bin/bash
# HBM traffic of the fused verify kernels (aux_bench verify row: RS(2,1) and RS(32,32) over a
# 64-segment batch): one PMC pass per counter group, kernel-trace only, then a stats pass.
# usage: tools/gpu_pmc_verify.sh <tag>
set -u
TAG=$1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$c" -o run -- \
    python -u tools/aux_bench.py --only verify > "$OUT/pmc_$c.log" 2>&1 ||
    { echo "pmc $c failed rc=$?"; tail -5 "$OUT/pmc_$c.log"; exit 1; }
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- \
  python -u tools/aux_bench.py --only verify > "$OUT/stats.log" 2>&1 ||
  { echo "stats failed rc=$?"; tail -5 "$OUT/stats.log"; exit 1; }
F=$(find "$OUT/pmc_FETCH_SIZE" -name "*counter_collection.csv" | head -1)
W=$(find "$OUT/pmc_WRITE_SIZE" -name "*counter_collection.csv" | head -1)
python tools/pmc_traffic.py "$F" "$W" k_verify21 "$OUT/traffic_verify21.json" $((64 * 3 * (8 << 20)))
python tools/pmc_traffic.py "$F" "$W" k_fft3232_verify "$OUT/traffic_fft3232_verify.json" \
  $((64 * 64 * (512 << 10)))
