#!/bin/bash
# records bench only
set -o pipefail
mkdir -p gpurun_out/r06b
timeout -k 10 500 python -u tools/records_bench.py --gib 8 --modes none,gpu,host,hybrid \
  --tails=-1,0,2,4 --reps 3 --stream 4 "$@" > gpurun_out/r06b/records_bench.jsonl 2>&1
rc=$?
cat gpurun_out/r06b/records_bench.jsonl
exit $rc
