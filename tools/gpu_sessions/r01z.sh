set -u
cd $GRAFT_REPO_ROOT; OUT=$PWD/gpurun_out/r01z; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --config 5 --steps 400 --warmup 5 --no-cpu-baseline > $OUT/c5.json 2>&1 || { tail $OUT/c5.json; exit 1; }
tail -1 $OUT/c5.json | cut -c1-200
for a in "--gib 4" "--gib 8" "--gib 32"; do
  timeout -k 10 300 python -u tools/e2e_bench.py $a --hash gpu > $OUT/e2e.json 2>&1 || { tail $OUT/e2e.json; exit 1; }
  echo "$a gpu: $(tail -1 $OUT/e2e.json)"
  timeout -k 10 300 python -u tools/e2e_bench.py $a --hash host > $OUT/e2e.json 2>&1 || { tail $OUT/e2e.json; exit 1; }
  echo "$a host: $(tail -1 $OUT/e2e.json)"
done
