set -u
cd $GRAFT_REPO_ROOT; OUT=$PWD/gpurun_out/r01o; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash tools/gpu_pmc.sh r01o 5 "EncCT<32, 32>, 4" 2147483648 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof5 -o run -- python -u bench.py --config 5 --no-cpu-baseline --steps 10 --warmup 2 > $OUT/prof5.log 2>&1 || { tail $OUT/prof5.log; exit 1; }
tail -1 $OUT/prof5.log
find $OUT/prof5 -name "*kernel_stats*" -exec cp {} $OUT/kernel_stats_c5.csv \;
cut -d, -f1-8 $OUT/kernel_stats_c5.csv | head -8
