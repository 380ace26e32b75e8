#!/bin/bash
# lane-pair tick: hash-queue tests on every tick kernel, then latency / throughput vs chains
set -o pipefail
mkdir -p gpurun_out/r06lp
timeout -k 10 600 python -u -m pytest tests/test_gpu_hashq.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r06lp/hashq_tests.log 2>&1 || { tail -30 gpurun_out/r06lp/hashq_tests.log; exit 1; }
tail -2 gpurun_out/r06lp/hashq_tests.log
for pf in 1 4 3; do
  timeout -k 10 200 python -u tools/sha_scale.py --blocks 2048 --stride 131136 --pf $pf \
    --chains 64,192,1024,4096,8192,16384,32768,65536 >> gpurun_out/r06lp/sha_scale.jsonl 2>&1 || exit 1
done
grep -v amdgpu gpurun_out/r06lp/sha_scale.jsonl
