#!/bin/bash
# round 5: is config 5's in-line gap the encode stream? in-line and standalone with the encode on
# a fresh torch stream ("new") or the current (null) stream ("current"), same box, interleaved
set -o pipefail
o=gpurun_out/r05/c5_gap2
mkdir -p $o
run() { # name, stream, args...
  local n=$1 st=$2; shift 2
  CESS_C5_STREAM=$st timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline > $o/$n.json 2> $o/$n.err || exit 1
  python - "$o/$n.json" "$n" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
c5 = (d.get("extra") or {}).get("config5")
print(sys.argv[2], d["ms_per_step"] if c5 is None else c5["ms_per_step"], flush=True)
PY
}
for r in a b; do
  run inline_new_$r new
  run inline_cur_$r current
  run sa384_new_$r new --config 5 --steps 384 --warmup 10
  run sa384_cur_$r current --config 5 --steps 384 --warmup 10
done
