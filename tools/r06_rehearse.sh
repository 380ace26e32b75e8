#!/bin/bash
# one-GPU rehearsal of the N-rank default line (N gloo ranks sharing GPU 0): wall time, the
# exchange legs, line_problems.   usage: tools/r06_rehearse.sh N TAG
set -o pipefail
N=${1:-2}; TAG=${2:-a}
o=gpurun_out/r06r_$TAG
mkdir -p $o
t0=$(date +%s.%N)
CESS_DIST_BACKEND=gloo CESS_DEVICE=0 timeout -k 10 560 python -u bench.py --gpus $N \
  > $o/bench_gpus${N}_gloo_one_gpu.json 2> $o/bench_gpus${N}_gloo_one_gpu.err
rc=$?
t1=$(date +%s.%N)
echo "{\"wall_s\": $(python -c "print(round($t1-$t0,1))"), \"rc\": $rc}" > $o/wall.json
cat $o/wall.json
tail -c 400 $o/bench_gpus${N}_gloo_one_gpu.err
N=$N TAG=$TAG python - <<'P'
import json, os, bench
o = f"gpurun_out/r06r_{os.environ['TAG']}/bench_gpus{os.environ['N']}_gloo_one_gpu.json"
d = json.loads(open(o).read().strip().splitlines()[-1])
print(sorted(d["extra"].keys()))
for k in ("degraded_gather", "wide_degraded_gather", "degraded_gather_cabi"):
    print(k, json.dumps(d["extra"].get(k))[:600])
print("line_problems", bench.line_problems(d))
P
exit $rc
