#!/bin/bash
# Round-3 checkpoint on HEAD: full GPU suite + smoke, the default bench line, rocprof kernel stats of
# the default line and of config 6 (32 random erasures: k_fftdec_d; 8: k_fftdec_m), the config-6
# sweep over erasure counts. Stops at the first failure.
# usage (GPU box): bash tools/gpu_round3_final.sh <tag>
set -u
TAG=${1:-r03s3}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu_tests.sh "$TAG" || exit 1
grep -q " passed" "$OUT/pytest_gpu.log" && ! grep -q " failed" "$OUT/pytest_gpu.log" || { echo "GPU tests failed"; exit 1; }
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
tail -c 300 "$OUT/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c2" -o run -- \
  python -u bench.py --no-cpu-baseline --no-extra > "$OUT/prof_c2.out" 2> "$OUT/prof_c2.err" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c6" -o run -- \
  python -u bench.py --config 6 --erasures 32 --no-cpu-baseline --steps 50 --warmup 5 \
  > "$OUT/prof_c6.out" 2> "$OUT/prof_c6.err" || exit 1
for e in 5 8 12 16 20 24 32; do  # config 6 by erasure count, the library's own pick
  timeout -k 10 120 python -u bench.py --config 6 --erasures $e --steps 50 --warmup 30 \
    --no-cpu-baseline >> "$OUT/c6_sweep.jsonl" 2>> "$OUT/c6_sweep.err" || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c6e8" -o run -- \
  python -u bench.py --config 6 --erasures 8 --no-cpu-baseline --steps 50 --warmup 30 \
  > "$OUT/prof_c6e8.out" 2> "$OUT/prof_c6e8.err" || exit 1
echo done
