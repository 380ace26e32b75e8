#!/bin/bash
# Variant sweep of the compile-time kernel on one GPU: bench lines to gpurun_out/<tag>/sweep.jsonl
set -u
TAG=${1:-sweep}; shift || true
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for cfg in "$@"; do
  for v in -1 0 1 2 3 4 5; do
    timeout -k 10 120 python -u bench.py --config "$cfg" --variant "$v" --no-cpu-baseline --no-extra \
      --steps 100 --warmup 10 > "$OUT/v.json" 2> "$OUT/v.err"
    rc=$?
    if [ $rc -ne 0 ]; then echo "variant $v config $cfg rc=$rc"; tail -3 "$OUT/v.err"; exit $rc; fi
    python -c "import json,sys; d=json.load(open('$OUT/v.json')); print(json.dumps({'config':$cfg,'variant':$v,'value':d['value'],'launch_ms':d['roofline']['launch_ms'],'frac':d['roofline']['frac']}))" | tee -a "$OUT/sweep.jsonl"
  done
done
