#!/bin/bash
# Quad / pair exchanges through DPP (product) or the LDS crossbar (ds_swizzle): the forms tests,
# then interleaved A/B of the derivative decoder (-1, 73 everywhere, 75 IFFT + derivative, 77 IFFT)
# at 20 and 32 erasures and of the syndrome-row decoder (-1, 79..82) at 5, 8 and 16.
set -u
TAG=${1:-r04_swz3}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "fftdec_d_forms or fftdec_m_forms" > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"
if [ $rc -ne 0 ]; then echo "tests rc=$rc"; exit $rc; fi
for e in 32 20; do
  timeout -k 10 200 python -u bench.py --config 6 --erasures $e --fftdec-mode 2 --sweep=-1,73,75,77 --steps 40 --warmup 30 > "$OUT/d_e$e.log" 2>&1 || exit $?
  echo "e=$e d"; grep '^{' "$OUT/d_e$e.log"
done
for e in 5 8 16; do
  timeout -k 10 200 python -u bench.py --config 6 --erasures $e --fftdec-mode 1 --sweep=-1,79,80,81,82 --steps 40 --warmup 30 > "$OUT/m_e$e.log" 2>&1 || exit $?
  echo "e=$e m"; grep '^{' "$OUT/m_e$e.log"
done
