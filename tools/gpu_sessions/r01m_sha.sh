set -u
cd $GRAFT_REPO_ROOT; OUT=$PWD/gpurun_out/r01m; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "sha256" -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
for mode in 1 2; do
  timeout -k 10 200 python -u bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline --sha-mode $mode > $OUT/c5_mode$mode.json 2>&1 || { tail $OUT/c5_mode$mode.json; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/c5_mode$mode.json').read().strip().splitlines()[-1]);print($mode, d['value'], d['sha256'])"
done
for mode in 1 2; do
  timeout -k 10 200 python -u bench.py --config 5 --segments 1024 --steps 2 --warmup 1 --no-cpu-baseline --sha-mode $mode > $OUT/c5big_mode$mode.json 2>&1 || { tail $OUT/c5big_mode$mode.json; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/c5big_mode$mode.json').read().strip().splitlines()[-1]);print('big', $mode, d['value'], d['sha256'])"
done
