set -u
cd $GRAFT_REPO_ROOT; OUT=$PWD/gpurun_out/r01zh; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_hashq.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for g in 8 12 16 64; do
  echo -n "--gib $g gpu: " >> $OUT/e2e.txt
  timeout -k 10 200 python -u tools/e2e_bench.py --gib $g --hash gpu >> $OUT/e2e.txt 2>$OUT/e2e.err || { tail $OUT/e2e.err; exit 1; }
done
cat $OUT/e2e.txt
timeout -k 10 300 python -u bench.py --config 5 --steps 100 --warmup 10 --no-cpu-baseline > $OUT/c5.json 2>$OUT/c5.err || { tail $OUT/c5.err; exit 1; }
tail -c 1500 $OUT/c5.json
