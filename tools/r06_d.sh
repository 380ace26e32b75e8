#!/bin/bash
# lane-refill host SHA: probe + records bench (host, hybrid) at depth 3/4
set -o pipefail
mkdir -p gpurun_out/r06d
timeout -k 10 120 python -u tools/host_sha_probe.py --threads 8,16 --mib 1024 --reps 2 > gpurun_out/r06d/host_sha_probe.jsonl 2>&1 || exit 1
for cfg in "--depth 3" "--depth 4" "--depth 4 --window 32"; do
  echo "== $cfg" >> gpurun_out/r06d/records.jsonl
  timeout -k 10 200 python -u tools/records_bench.py --gib 8 --modes host,hybrid --tails=-1,0 \
    --reps 3 --stream 4 $cfg >> gpurun_out/r06d/records.jsonl 2>&1 || exit 1
done
grep -v "probe\|amdgpu.ids" gpurun_out/r06d/host_sha_probe.jsonl
grep -v amdgpu.ids gpurun_out/r06d/records.jsonl
