#!/bin/bash
# One-wave tick occupancy variants (CEC_HQOPT_TICK 3 = 100 VGPRs / 5 waves, 5 = pinned schedule
# 74 VGPRs / 6 waves, 6 = pinned + 8 waves requested (64 VGPRs, 48 B scratch), 7 = unpinned + 6
# waves (80 VGPRs, 112 B scratch)): tick throughput in the throughput regime, then config 5's step.
# The variants (k_sha256_tick1<0>, k_sha256_tick1_occ<D, W>) existed for this measurement only
# (profiles/r06/tick_occupancy/): none was faster, and they were removed.
set -o pipefail
OUT=gpurun_out/r06occ; rm -rf $OUT; mkdir -p $OUT
for pf in 3 5 6 7; do
  timeout -k 10 120 python -u tools/sha_scale.py --blocks 128 --stride 8192 --pf $pf \
    --chains 65536,131072,262144,393216 > $OUT/scale_$pf.jsonl 2>&1 || exit 1
  echo "== tick $pf"; grep -v amdgpu $OUT/scale_$pf.jsonl
done
for pf in 3 5 6 3 5 6; do
  timeout -k 10 200 python -u bench.py --config 5 --tick-pf $pf --no-cpu-baseline > $OUT/c5_$pf.log 2>&1 || exit 1
  echo "== config 5 tick $pf"; grep '^{' $OUT/c5_$pf.log | python -c "
import sys, json
d = json.loads(sys.stdin.read().splitlines()[-1]); print(d['ms_per_step'], d.get('sha256', {}).get('roofline', {}).get('frac'))"
done
