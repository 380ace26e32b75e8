#!/bin/bash
# Host SHA x16: software prefetch distance A/B (CEC_HOST_SHA_PREFETCH bytes ahead per lane; the
# knob existed for this measurement only and was removed after it: profiles/r06/prefetch_ab/).
set -o pipefail
OUT=gpurun_out/r06pf; rm -rf $OUT; mkdir -p $OUT
for pf in 0 256 512 1024 2048 0; do
  CEC_HOST_SHA_PREFETCH=$pf timeout -k 10 100 python tools/host_sha_probe.py --threads 1,16 --mib 4096 --reps 2 > $OUT/probe_$pf.jsonl 2>&1 || exit 1
  echo "== prefetch $pf"; grep '"x16"' $OUT/probe_$pf.jsonl | grep -v probe
done
for pf in 0 512 0 512; do
  CEC_HOST_SHA_PREFETCH=$pf timeout -k 10 150 python -u tools/records_bench.py --gib 8 --modes host --reps 3 > $OUT/rb_$pf.jsonl 2>&1 || exit 1
  echo "== records host prefetch $pf"; grep best_GBps $OUT/rb_$pf.jsonl | cut -c1-200
done
