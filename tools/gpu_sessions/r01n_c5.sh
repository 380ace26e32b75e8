set -u
cd $GRAFT_REPO_ROOT; OUT=$PWD/gpurun_out/r01n; mkdir -p $OUT
timeout -k 10 200 python -u bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/c5.json 2>&1 || { tail $OUT/c5.json; exit 1; }
tail -1 $OUT/c5.json
timeout -k 10 200 python -u bench.py --config 5 --segments 1024 --steps 4 --warmup 1 --no-cpu-baseline > $OUT/c5big.json 2>&1 || { tail $OUT/c5big.json; exit 1; }
tail -1 $OUT/c5big.json
