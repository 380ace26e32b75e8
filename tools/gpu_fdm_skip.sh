#!/bin/bash
# k_fftdec_m's skip of coset-A slots with no position read: the forms test, then the product (-1)
# against tuning form 86 (no skip), one form per process, alternating, on consecutive-erasure
# patterns and on random ones.
set -u
TAG=${1:-r04_fdmskip}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "fftdec_m_forms or fftdec_d_forms or both_decoders" > "$OUT/tests.log" 2>&1
rc=$?; tail -2 "$OUT/tests.log"
if [ $rc -ne 0 ]; then echo "tests rc=$rc"; exit $rc; fi
: > "$OUT/runs.jsonl"
one() {  # one <erasures> <run flag or ''> <variant>
  timeout -k 10 120 python -u bench.py --config 6 --erasures $1 $2 --fftdec-mode 1 --variant $3 \
    --steps 50 --warmup 30 --no-cpu-baseline --no-extra > "$OUT/one.log" 2>&1 || { tail -5 "$OUT/one.log"; exit 1; }
  grep '^{' "$OUT/one.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'e': $1, 'run': '$2' != '', 'variant': $3, 'ms': d['roofline']['launch_ms']}))" | tee -a "$OUT/runs.jsonl"
}
for rep in 1 2 3; do
  for v in -1 86; do one 8 --erasure-run $v; done
  for v in -1 86; do one 16 --erasure-run $v; done
  for v in -1 86; do one 8 "" $v; done
done
