#!/bin/bash
# Round profile session: default bench line + rocprof kernel stats per BASELINE config, C host
# pipeline end-to-end rates, SQ counters of the RS(32,32) encode. Stops at the first crash/timeout.
# usage: tools/gpu_profile.sh <tag>
set -u
TAG=${1:-r02}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # run <name> <timeout> cmd...
  local name=$1 tmo=$2; shift 2
  echo "== $name"
  timeout -k 10 "$tmo" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  tail -c 400 "$OUT/$name.out"; echo
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "$OUT/$name.err"; exit $rc; fi
}
run bench_c2 300 python -u bench.py
for c in 2 3 5; do
  run prof_c$c 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c$c" -o run -- \
    python -u bench.py --config $c --no-cpu-baseline --no-extra --steps 100 --warmup 10
done
run bench_c3 300 python -u bench.py --config 3 --cpu-seconds 4
run bench_c5 300 python -u bench.py --config 5 --steps 400 --warmup 20 --cpu-seconds 4
run bench_c4 300 python -u bench.py --config 4 --steps 5 --warmup 2 --cpu-seconds 4
run pmc_sq_fft 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d "$OUT/pmc_sq_fft" -o run -- \
  python -u bench.py --config 5 --sweep=-1 --steps 2 --warmup 1
gcc -O2 -pthread tests/native/pipeline_e2e.c -Iinclude -Lcess_amd -lcessec -Loracle/build -loracle \
  -Wl,-rpath,$PWD/cess_amd:$PWD/oracle/build -o /tmp/pe2e || exit 1
for args in "2 1 8388608 1024 64 3 0 16 64 1073741824" "2 1 8388608 1024 64 3 1 32 64 1073741824" \
            "2 1 8388608 4096 64 3 1 32 64 1073741824" "32 32 524288 1024 64 3 1 32 64 1073741824"; do
  run e2e_$(echo $args | tr ' ' '_') 300 /tmp/pe2e $args
done
find "$OUT" -name "*kernel_stats.csv" | while read f; do cp "$f" "$OUT/$(basename $(dirname $f))_kernel_stats.csv"; done
echo done
