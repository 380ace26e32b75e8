#!/bin/bash
# The pipeline's H2D / D2H copies run as __amd_rocclr_copyBuffer blit kernels (HSA_ENABLE_SDMA=1
# changes nothing: profiles/r06/sdma/), whose waves take issue slots from the hash ticks beside
# them. Does capping the blit kernels' workgroups (DEBUG_CLR_LIMIT_BLIT_WG) free the ticks
# without slowing the copies? records_bench: no hashing, hybrid lone file, four-file stream.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06blitwg; rm -rf $OUT; mkdir -p $OUT
run() {  # name [wg]
  if [ -n "${2:-}" ]; then export DEBUG_CLR_LIMIT_BLIT_WG=$2; else unset DEBUG_CLR_LIMIT_BLIT_WG; fi
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
for rep in 1 2; do run def_$rep; run wg64_$rep 64; run wg16_$rep 16; done
