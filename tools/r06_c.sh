#!/bin/bash
# records bench sweep: host SHA form x depth x window
set -o pipefail
mkdir -p gpurun_out/r06c
for cfg in "--form 2 --depth 3" "--form 4 --depth 3" "--form 2 --depth 4" "--form 4 --depth 4" "--form 4 --depth 4 --window 32" "--form 2 --depth 4 --window 32"; do
  tag=$(echo $cfg | tr -d ' -')
  echo "== $cfg" >> gpurun_out/r06c/records_sweep.jsonl
  timeout -k 10 200 python -u tools/records_bench.py --gib 8 --modes host,hybrid --tails=-1,0 \
    --reps 3 --stream 4 $cfg >> gpurun_out/r06c/records_sweep.jsonl 2>&1 || exit 1
done
cat gpurun_out/r06c/records_sweep.jsonl | grep -v amdgpu.ids
