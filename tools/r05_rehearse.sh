#!/bin/bash
# round 5: one-GPU rehearsals of the N = 2 and N = 4 default lines (gloo ranks sharing GPU 0)
# usage: tools/r05_rehearse.sh [suffix] [world sizes...]   (default: b, 2 4)
set -o pipefail
o=gpurun_out/r05
mkdir -p $o
sfx=${1:-b}
shift
sizes=${*:-2 4}
for n in $sizes; do
  CESS_DIST_BACKEND=gloo CESS_DEVICE=0 timeout -k 10 600 python -u bench.py --gpus $n \
    > $o/bench_gpus${n}_gloo_one_gpu_${sfx}.json 2> $o/bench_gpus${n}_gloo_one_gpu_${sfx}.err || exit 1
done
