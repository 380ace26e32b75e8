#!/bin/bash
# round 5: PMC HBM bytes of the 64 GiB (4096-segment) RS(2,1) encode launch of extra.config4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out/r05/pmc_c4; mkdir -p "$OUT"
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$c" -o run -- \
    python -u bench.py --config 2 --segments 4096 --no-cpu-baseline --no-extra --steps 3 \
    --warmup 1 > "$OUT/pmc_$c.log" 2>&1 || { echo "pmc $c failed rc=$?"; tail -5 "$OUT/pmc_$c.log"; exit 1; }
done
F=$(find "$OUT/pmc_FETCH_SIZE" -name "*counter_collection.csv" | head -1)
W=$(find "$OUT/pmc_WRITE_SIZE" -name "*counter_collection.csv" | head -1)
python tools/pmc_traffic.py "$F" "$W" "EncCT<2, 1>" "$OUT/traffic_c4.json" 103079215104
