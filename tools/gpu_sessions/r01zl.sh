set -u
cd $GRAFT_REPO_ROOT; OUT=$PWD/gpurun_out/r01zl; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2 -o c2 -- python -u bench.py > $OUT/c2.json 2>$OUT/c2.err || { tail $OUT/c2.err; exit 1; }
tail -1 $OUT/c2.json | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o c3 -- python -u bench.py --config 3 --no-cpu-baseline > $OUT/c3.json 2>$OUT/c3.err || { tail $OUT/c3.err; exit 1; }
tail -1 $OUT/c3.json | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5 -o c5 -- python -u bench.py --config 5 --steps 100 --warmup 5 --no-cpu-baseline > $OUT/c5.json 2>$OUT/c5.err || { tail $OUT/c5.err; exit 1; }
tail -1 $OUT/c5.json | cut -c1-200
find $OUT -name "*stats*" | head
