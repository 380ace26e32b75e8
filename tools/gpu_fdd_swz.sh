#!/bin/bash
# k_fftdec_d's quad exchanges: DPP (product) against the LDS crossbar (tuning variant 73). The forms
# test, then the interleaved A/B at 16, 24, 32 erasures (config 6, derivative decoder forced),
# with the crossbar in every phase (73) or in some (74..78).
set -u
TAG=${1:-r04_swz}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "fftdec_d_forms" > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"
if [ $rc -ne 0 ]; then echo "tests rc=$rc"; exit $rc; fi
# variants: -1 DPP everywhere (product), 73 the crossbar everywhere, 74..78 in some phases
for e in 32 24 16; do
  timeout -k 10 200 python -u bench.py --config 6 --erasures $e --fftdec-mode 2 --sweep=-1,73,74,75,76,77,78 --steps 30 --warmup 30 > "$OUT/ab_e$e.log" 2>&1 || exit $?
  grep '^{' "$OUT/ab_e$e.log"
done
