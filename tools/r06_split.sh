#!/bin/bash
# Host SHA pool lane split A/B: the wide / narrow split (this tree) against the previous policy
# (tools/ab/libcessec_prev.so: fill 16 lanes when chains are plentiful, else a fair SHA-NI
# share), alternating: the x16 pool at 64..576 chains, then the records placements. The split
# (and tools/ab/) existed for this measurement only (profiles/r06/lane_split_ab/, the last of
# three variants): it was within the box's run-to-run spread, and the previous policy stayed.
set -o pipefail
OUT=gpurun_out/r06split; rm -rf $OUT; mkdir -p $OUT
for rep in 1 2 3; do
  for v in new prev; do
    if [ $v = prev ]; then L=tools/ab/libcessec_prev.so; else L=cess_amd/libcessec.so; fi
    for mib in 1024 4608; do
      timeout -k 10 100 python tools/host_sha_probe.py --lib $L --threads 16 --mib $mib --reps 2 --forms 4 > $OUT/probe_${v}_${mib}_$rep.jsonl 2>&1 || exit 1
    done
    CESS_EC_LIB=$PWD/$L timeout -k 10 150 python -u tools/records_bench.py --gib 8 --modes host,hybrid --reps 3 --stream 4 > $OUT/rb_${v}_$rep.jsonl 2>&1 || exit 1
    echo "== $v $rep"
    grep -h '"x16"' $OUT/probe_${v}_*_$rep.jsonl | grep -v probe | python -c "
import sys, json
print(' '.join(str(json.loads(l)['GBps']) for l in sys.stdin))"
    grep -h "best_GBps\|records_stream" $OUT/rb_${v}_$rep.jsonl | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['mode'], d.get('best_GBps'), d.get('seconds'), d.get('GBps'), d.get('cpu_seconds'))"
  done
done
