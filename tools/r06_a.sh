#!/bin/bash
# round 6, first GPU pass: pipeline tests (all hash modes) + records bench of the placements
set -o pipefail
mkdir -p gpurun_out/r06a
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_host_sha.py -x -v \
  --timeout 240 --timeout-method thread > gpurun_out/r06a/pipeline_tests.log 2>&1 || { tail -30 gpurun_out/r06a/pipeline_tests.log; exit 1; }
tail -3 gpurun_out/r06a/pipeline_tests.log
timeout -k 10 400 python -u tools/records_bench.py --gib 8 --modes none,gpu,host,hybrid \
  --tails=-1,0,2,4 --reps 3 --stream 4 > gpurun_out/r06a/records_bench.jsonl 2>&1
rc=$?
cat gpurun_out/r06a/records_bench.jsonl
exit $rc
