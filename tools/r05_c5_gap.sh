#!/bin/bash
# round 5: config 5's in-line leg (default line) against standalone runs, same box, interleaved
set -o pipefail
o=gpurun_out/r05/c5_gap
mkdir -p $o
run() { # name, args...
  local n=$1; shift
  timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline > $o/$n.json 2> $o/$n.err || exit 1
  python - "$o/$n.json" "$n" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
c5 = (d.get("extra") or {}).get("config5")
print(sys.argv[2], d["ms_per_step"] if c5 is None else c5["ms_per_step"], flush=True)
PY
}
run sa400_a --config 5 --steps 400 --warmup 20
run inline_a
run sa100_a --config 5
run sa384_a --config 5 --steps 384 --warmup 10
run inline_b
run sa400_b --config 5 --steps 400 --warmup 20
