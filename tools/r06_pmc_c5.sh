#!/bin/bash
# config 5's shader clock under the hash ticks and the encode (GRBM_GUI_ACTIVE), one --pmc pass
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out/r06_pmc_c5; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVES --output-format csv \
  -d "$OUT/pmc_clock" -o run -- python -u bench.py --config 5 --no-cpu-baseline --no-extra \
  --steps 120 --warmup 10 > "$OUT/pmc_clock.log" 2>&1 || { echo "pmc failed rc=$?"; tail -5 "$OUT/pmc_clock.log"; exit 1; }
F=$(find "$OUT/pmc_clock" -name "*counter_collection.csv" | head -1)
python tools/pmc_clock.py "$F" "$OUT/pmc_c5_clock.json"
