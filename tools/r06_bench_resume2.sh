#!/bin/bash
# The bench line's host_e2e with the opt-in resume after the state ring change (4 nd state slots
# instead of one per device slot), on and off; the pipeline tests (resume path included) first.
# The ring variant existed for this measurement only (no change: profiles/r06/bench_resume_trace/)
# and was reverted. Run again with the tick slack for resumed chains (pipeline.cpp, window - 4
# ticks per chain): profiles/r06/bench_resume_slack/.
set -o pipefail
OUT=gpurun_out/r06benchres2; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_pipeline.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for v in on off on; do
  if [ $v = on ]; then export CEC_PIPELINE_RESUME=1; else unset CEC_PIPELINE_RESUME; fi
  timeout -k 10 400 python -u bench.py --no-cpu-baseline > $OUT/bench_$v.log 2>&1 || exit 1
  echo "== $v"; grep '^{' $OUT/bench_$v.log | tail -1 | python -c "
import sys, json
d = json.loads(sys.stdin.read()); h = d['extra']['host_e2e']
print({k: (h[k].get('node_GBps'), h[k].get('cpu_s', h[k].get('cpu_s_runs')), h[k].get('file_done_s')) for k in ('segment_lists_hybrid', 'records_stream')})"
done
