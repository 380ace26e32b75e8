#!/bin/bash
# Config-5 whole step with the encode and the hash ticks on equal vs prioritised streams.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/c5prio
for p in 0 1; do
  timeout -k 10 200 python -u bench.py --config 5 --steps 400 --warmup 20 --no-cpu-baseline \
    --prio $p > gpurun_out/c5prio/prio$p.json || exit 1
  python -c "import json; d=json.load(open('gpurun_out/c5prio/prio$p.json')); print('prio', $p, d['value'], d['ms_per_step'])"
done
