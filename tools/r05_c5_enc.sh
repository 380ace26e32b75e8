#!/bin/bash
# round 5: config 5's step with each RS(32,32) encode form of the tuning build: is the step (VALU
# bound by the hash ticks) faster with an encode that issues fewer VALU slots, even if slower alone?
set -o pipefail
o=gpurun_out/r05/c5_enc
mkdir -p $o
for r in a b; do
  for v in -1 21 11 13 3; do
    timeout -k 10 200 python -u bench.py --config 5 --steps 384 --warmup 10 --no-cpu-baseline \
      --variant $v > $o/v${v}_$r.json 2> $o/v${v}_$r.err || exit 1
    python - "$o/v${v}_$r.json" "$v" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("variant", sys.argv[2], "step_ms", d["ms_per_step"], "encode_ms", d["sha256"]["encode_ms"], flush=True)
PY
  done
done
