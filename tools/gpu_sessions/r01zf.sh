set -u
cd $GRAFT_REPO_ROOT; OUT=$PWD/gpurun_out/r01zf; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "segment_list or auto" -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for g in 4 8 16; do
  echo -n "--gib $g host: " >> $OUT/e2e.txt
  timeout -k 10 200 python -u tools/e2e_bench.py --gib $g --hash host >> $OUT/e2e.txt 2>$OUT/e2e.err || { tail $OUT/e2e.err; exit 1; }
done
cat $OUT/e2e.txt
