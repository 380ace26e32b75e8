#!/bin/bash
# k_fftdec_dp (pipelined, default) vs k_fftdec_d (one block per wave, tuning variant 70) vs the
# pipelined kernel with LDS-DMA staging (71): the fftdec GPU tests, then interleaved A/B sweeps.
set -u
TAG=${1:-r04_fdd}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
step() {
  local name=$1 tmo=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  if grep -q "illegal memory access\|Memory access fault\|HSA_STATUS_ERROR" "$OUT/$name.log"; then
    echo "stopping after $name: GPU fault"; exit 3; fi
  return 0
}
step tests 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "fftdec or wide or host_api or dist or partial or repair"
for e in 32 24 16; do
  step ab_e$e 120 python -u bench.py --config 6 --erasures $e --fftdec-mode 2 --sweep=-1,70,71 --steps 20 --warmup 30
done
step c6_e32 120 python -u bench.py --config 6 --erasures 32 --no-cpu-baseline
echo done
