#!/bin/bash
# round 5, GPU call 2: C-ABI dist tests (stand-in world 2..8 and world 1), then the config-5 A/B
# across library builds, then the one-GPU gloo rehearsal of the N = 2 default line
set -o pipefail
o=gpurun_out/r05
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_dist_standin.py "tests/test_gpu_multi.py" -m gpu -x -v \
  --timeout 200 --timeout-method thread > $o/dist_tests.log 2>&1 || exit 1
bash tools/c5_ab.sh || exit 1
CESS_DIST_BACKEND=gloo CESS_DEVICE=0 timeout -k 10 600 python -u bench.py --gpus 2 \
  > $o/bench_gpus2_gloo_one_gpu_a.json 2> $o/bench_gpus2_gloo_one_gpu_a.err || exit 1
