#!/bin/bash
# Kernel trace of the default bench line with the opt-in hybrid resume (the stream leg there ran
# at 25-26 GB/s against 41-42 standalone).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06bresprof; rm -rf $OUT; mkdir -p $OUT
CEC_PIPELINE_RESUME=1 timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $OUT -o b -- python3 -u bench.py --no-cpu-baseline > $OUT/bench.log 2>&1 || exit 1
grep '^{' $OUT/bench.log | tail -1 | python -c "
import sys, json
d = json.loads(sys.stdin.read()); h = d['extra']['host_e2e']
print({k: (h[k].get('node_GBps'), h[k].get('file_done_s')) for k in ('segment_lists_hybrid', 'records_stream')})"
ls -la $OUT/*.csv
