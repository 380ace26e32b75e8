#!/bin/bash
# Records placements with the pipeline's wait trace and the host SHA pool's busy time.
set -o pipefail
OUT=gpurun_out/r06trace; rm -rf $OUT; mkdir -p $OUT
CEC_PIPELINE_TRACE=1 timeout -k 10 200 python -u tools/records_bench.py --gib 8 --modes host,hybrid --reps 3 --stream 4 > $OUT/rb.jsonl 2>&1 || exit 1
grep -v "destroy\|amdgpu" $OUT/rb.jsonl | cut -c1-420
