#!/bin/bash
# round 5: config 3 (RS(2,1) rebuild, erased = seg mod 3) with the tagged-list mixed kernel
# (product, -1) against tuning variant 90 (erasures in the kernel arguments, natural order), the
# uniform pattern and the encode beside them; interleaved, one process each
set -o pipefail
o=gpurun_out/r05/c3_kargs
mkdir -p $o
run() {
  local n=$1; shift
  timeout -k 10 200 python -u bench.py "$@" --no-cpu-baseline --no-extra --steps 200 \
    > $o/$n.json 2> $o/$n.err || exit 1
  python - "$o/$n.json" "$n" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[2], d["roofline"]["launch_ms"], d["roofline"]["frac"], flush=True)
PY
}
for r in a b c; do
  run c3_prod_$r --config 3
  run c3_v90_$r --config 3 --variant 90
  run c3_e0_$r --config 3 --erase 0
  run c2_$r --config 2
done
