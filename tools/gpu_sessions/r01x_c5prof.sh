set -u
cd $GRAFT_REPO_ROOT; OUT=$PWD/gpurun_out/r01x; mkdir -p $OUT
export TMPDIR=/tmp
for w in 16 64; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_w$w -o c5 -- python -u bench.py --config 5 --window $w --hash-stream 0 --steps 100 --warmup 5 --no-cpu-baseline > $OUT/rocprof_c5_w$w.log 2>&1 || { tail $OUT/rocprof_c5_w$w.log; exit 1; }
tail -1 $OUT/rocprof_c5_w$w.log | cut -c1-300
done
