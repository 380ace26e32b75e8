#!/bin/bash
# The pipeline's parity D2H shows up as __amd_rocclr_copyBuffer blit kernels beside the hash
# ticks. Is the box forcing blits (HSA_ENABLE_SDMA), and does the SDMA engine do better? The
# environment, records_bench's four-file hybrid stream with the default and HSA_ENABLE_SDMA=1
# alternating, then each under a kernel trace (copy kernels counted).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06sdma; rm -rf $OUT; mkdir -p $OUT
env | grep -i -E "sdma|^hsa_|^hip_|^gpu_|^roc" | sort > $OUT/env.txt; cat $OUT/env.txt
run() {  # name [sdma]
  if [ -n "${2:-}" ]; then export HSA_ENABLE_SDMA=$2; else unset HSA_ENABLE_SDMA; fi
  timeout -k 10 200 python -u tools/records_bench.py --gib 8 --modes none,hybrid --reps 3 --stream 4 --pieces > $OUT/rb_$1.jsonl 2>&1 || exit 1
  echo "== $1"; python - $OUT/rb_$1.jsonl <<'P'
import sys, json
for l in open(sys.argv[1]):
    if not l.startswith('{'): continue
    d = json.loads(l)
    if 'best_GBps' in d: print(d['mode'], 'best', d['best_GBps'], d['seconds'])
    elif 'GBps' in d: print('stream', d.get('GBps'), d.get('cpu_seconds'))
P
}
for rep in 1 2; do run def_$rep; run sdma1_$rep 1; done
for v in def sdma1; do
  if [ $v = sdma1 ]; then export HSA_ENABLE_SDMA=1; else unset HSA_ENABLE_SDMA; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$v -o rb -- python3 -u tools/records_bench.py --gib 8 --modes hybrid --reps 1 --stream 4 --pieces > $OUT/prof_$v.log 2>&1 || exit 1
  echo "== prof $v"; grep -h -o '"[^"]*copyBuffer[^"]*",[0-9]*' $OUT/prof_$v/*/rb_kernel_stats.csv $OUT/prof_$v/rb_kernel_stats.csv 2>/dev/null | head -3 || true
done
