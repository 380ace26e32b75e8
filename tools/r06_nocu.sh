#!/bin/bash
# (experiment) the pipeline's batch copies as hipMemcpyDeviceToDeviceNoCU (CEC_PIPELINE_NOCU):
# do they leave the CUs (no copyBuffer kernels) and free the ticks? The pipeline tests with it
# on first (records and fragments against the oracle), then records_bench alternating, then a
# kernel trace with it on.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06nocu; rm -rf $OUT; mkdir -p $OUT
CEC_PIPELINE_NOCU=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_pipeline.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
run() {  # name [on]
  if [ -n "${2:-}" ]; then export CEC_PIPELINE_NOCU=1; else unset CEC_PIPELINE_NOCU; fi
  timeout -k 10 200 python -u tools/records_bench.py --gib 8 --modes none,gpu,hybrid --reps 3 --stream 4 --pieces > $OUT/rb_$1.jsonl 2>&1 || exit 1
  echo "== $1"; python - $OUT/rb_$1.jsonl <<'P'
import sys, json
for l in open(sys.argv[1]):
    if not l.startswith('{'): continue
    d = json.loads(l)
    if 'best_GBps' in d: print(d['mode'], 'best', d['best_GBps'], d['seconds'])
    elif 'GBps' in d: print('stream', d['mode'], d.get('GBps'), d.get('cpu_seconds'))
P
}
for rep in 1 2; do run nocu_$rep 1; run def_$rep; done
export CEC_PIPELINE_NOCU=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o rb -- python3 -u tools/records_bench.py --gib 8 --modes hybrid --reps 1 --stream 4 --pieces > $OUT/prof.log 2>&1 || exit 1
echo "== prof nocu"; head -6 $OUT/prof/rb_kernel_stats.csv | cut -c1-150
# The toggle (pipeline.cpp, CEC_PIPELINE_NOCU) changed nothing and was reverted: the copies stayed
# copyBuffer kernels (profiles/r06/nocu/).
