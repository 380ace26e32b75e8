#!/bin/bash
# Host SHA pool with the tail spill: probe (288 x 16 MiB chains on 16 threads) and the records
# placements on an 8 GiB file, with the process's CPU seconds per run.
set -o pipefail
OUT=gpurun_out/r06spill; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 150 python tools/host_sha_probe.py --threads 16 --mib 4608 --reps 2 > $OUT/probe.jsonl 2>&1 || exit 1
timeout -k 10 250 python -u tools/records_bench.py --gib 8 --modes none,host,hybrid --reps 3 --stream 4 > $OUT/rb.jsonl 2>&1 || exit 1
grep -v "probe\|amdgpu\|destroy" $OUT/probe.jsonl $OUT/rb.jsonl
