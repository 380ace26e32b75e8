#!/bin/bash
# round 6 check: GPU suite + smoke, then the retrieval line at the new defaults
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r06check}
bash tools/gpu_tests.sh $TAG || exit $?
OUT=gpurun_out/$TAG
timeout -k 10 300 python -u tools/retrieve_bench.py --gib 4 > $OUT/retrieve_lost.jsonl 2>&1 || exit 1
timeout -k 10 300 python -u tools/retrieve_bench.py --gib 4 --intact > $OUT/retrieve_intact.jsonl 2>&1 || exit 1
grep GBps $OUT/retrieve_*.jsonl
