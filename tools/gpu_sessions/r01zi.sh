set -u
cd $GRAFT_REPO_ROOT; OUT=$PWD/gpurun_out/r01zi; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for c in 3 2 3 2; do
  timeout -k 10 200 python -u bench.py --config $c --steps 100 --warmup 10 --no-cpu-baseline > $OUT/b.json 2>$OUT/b.err || { tail $OUT/b.err; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]);print('config $c', d['value'], d['roofline']['achieved'], d['roofline']['launch_ms'], d['config']['kernel'])"
done
