#!/bin/bash
# lane-pair SHA kernels: SHA / hash-queue / pipeline / repair GPU tests, the latency sweep with the
# new auto threshold, the f2 / f4 rows (repair check, fillers)
set -o pipefail
mkdir -p gpurun_out/r06lp2
timeout -k 10 700 python -u -m pytest tests/test_gpu_hashq.py tests/test_gpu_parity.py tests/test_gpu_pipeline.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r06lp2/tests.log 2>&1 || { tail -30 gpurun_out/r06lp2/tests.log; exit 1; }
tail -2 gpurun_out/r06lp2/tests.log
timeout -k 10 200 python -u tools/sha_scale.py --blocks 2048 --stride 131136 --pf 0 \
    --chains 64,1024,16384,32768,49152,65536,131072 > gpurun_out/r06lp2/sha_scale_auto.jsonl 2>&1 || exit 1
timeout -k 10 300 python -u tools/aux_bench.py > gpurun_out/r06lp2/aux_bench.jsonl 2>&1 || exit 1
grep -v amdgpu gpurun_out/r06lp2/sha_scale_auto.jsonl gpurun_out/r06lp2/aux_bench.jsonl
