set -u
cd $GRAFT_REPO_ROOT; OUT=$PWD/gpurun_out/r01zk; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "ct_variants_identical" -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for v in -1 17 18 -1 17 18; do
  timeout -k 10 200 python -u bench.py --config 5 --variant $v --window 1 --hash-stream 0 --steps 100 --warmup 10 --no-cpu-baseline --no-extra > $OUT/b.json 2>$OUT/b.err || { tail $OUT/b.err; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]);print('c5 variant $v', d['roofline']['achieved'], d['roofline']['launch_ms'])" | tee -a $OUT/ab.txt
done
