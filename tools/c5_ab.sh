#!/bin/bash
# Same-box A/B of BASELINE config 5 (RS(32,32) encode + SHA-256 hash queue) across library builds:
# HEAD and the historical commits staged under tools/bisect/<commit>/ (their own bench.py, Python
# wrappers and product libcessec.so). Interleaved, two rounds, one process per run.
set -o pipefail
out=gpurun_out/r05/c5_ab
mkdir -p $out
for r in 1 2; do
  for c in HEAD c2659ea 970728f ef00dfb; do
    d=.; [ "$c" != HEAD ] && d=tools/bisect/$c
    (cd $d && timeout -k 10 150 python -u bench.py --config 5 --steps 400 --warmup 20 --no-cpu-baseline) \
      > $out/${c}_$r.json 2> $out/${c}_$r.err || exit 1
    echo "$c $r $(python -c "import json;d=json.load(open('$out/${c}_$r.json'));print(d['ms_per_step'])")"
  done
done
