#!/bin/bash
# Derivative-decoder forms, second pass: the forms test, the interleaved A/B at 32 erasures, then
# SQ counters of each form (tools/gpu_pmc_fdd.sh).
set -u
TAG=${1:-r04_fdd3}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "fftdec_d_forms or both_decoders" > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"
if [ $rc -ne 0 ]; then echo "tests rc=$rc"; exit $rc; fi
timeout -k 10 120 python -u bench.py --config 6 --erasures 32 --fftdec-mode 2 --sweep=-1,70,72 --steps 20 --warmup 30 > "$OUT/ab_e32.log" 2>&1 || exit $?
cat "$OUT/ab_e32.log" | grep '^{'
bash tools/gpu_pmc_fdd.sh "$TAG" "72"
