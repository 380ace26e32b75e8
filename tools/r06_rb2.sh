#!/bin/bash
set -o pipefail
OUT=gpurun_out/r06rb2; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 120 python tools/host_sha_probe.py --threads 16 --mib 2048 --reps 2 > $OUT/probe.jsonl 2>&1 || exit 1
timeout -k 10 250 python -u tools/records_bench.py --gib 8 --modes host,hybrid --tails=-1,0 --reps 3 --stream 4 > $OUT/rb.jsonl 2>&1 || exit 1
grep -v "probe\|amdgpu\|destroy" $OUT/probe.jsonl $OUT/rb.jsonl
