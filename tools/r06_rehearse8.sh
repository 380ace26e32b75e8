#!/bin/bash
# round 6: one-GPU rehearsal of the N = 8 default line (8 gloo ranks sharing GPU 0), wall time
set -o pipefail
o=gpurun_out/r06r
mkdir -p $o
t0=$(date +%s.%N)
CESS_DIST_BACKEND=gloo CESS_DEVICE=0 timeout -k 10 560 python -u bench.py --gpus 8 \
  > $o/bench_gpus8_gloo_one_gpu.json 2> $o/bench_gpus8_gloo_one_gpu.err
rc=$?
t1=$(date +%s.%N)
echo "{\"wall_s\": $(python -c "print(round($t1-$t0,1))"), \"rc\": $rc}" > $o/wall.json
cat $o/wall.json
tail -c 400 $o/bench_gpus8_gloo_one_gpu.err
python - <<'P'
import json
d=json.loads(open("gpurun_out/r06r/bench_gpus8_gloo_one_gpu.json").read().strip().splitlines()[-1])
print(sorted(d["extra"].keys()))
print(json.dumps(d["extra"].get("resources"), indent=0)[:3000])
P
exit $rc
