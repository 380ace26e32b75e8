#!/bin/bash
# HBM traffic of the config-6 rebuild (32 random erasures: k_fftdec_d): FETCH_SIZE and WRITE_SIZE
# in separate rocprofv3 --pmc passes (MI355X_MICROARCH.md HBM section), kernel-trace only.
# usage (GPU box): bash tools/gpu_pmc_c6.sh <tag>; then tools/pmc_traffic.py on the two csvs
set -u
TAG=${1:-pmc_c6}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d "$OUT/$c" -o run -- \
    python -u bench.py --config 6 --erasures 32 --no-cpu-baseline --no-extra --steps 5 --warmup 1 \
    > "$OUT/$c.log" 2>&1 || { echo "pmc $c failed"; tail -5 "$OUT/$c.log"; exit 1; }
  cp "$(find "$OUT/$c" -name '*counter_collection.csv' | head -1)" "$OUT/$c.csv"
done
echo done
