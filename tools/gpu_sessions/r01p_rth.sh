set -u
cd $GRAFT_REPO_ROOT; OUT=$PWD/gpurun_out/r01p; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "runtime_kernels or golden or per_segment or repair or degraded" -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for args in "--config 6 --rt-mode 0" "--config 6 --rt-mode 1" "--config 5 --generic --rt-mode 0" "--config 5 --generic --rt-mode 1" "--config 2 --generic --rt-mode 0" "--config 2 --generic --rt-mode 1"; do
  timeout -k 10 200 python -u bench.py $args --steps 10 --warmup 2 --no-cpu-baseline --no-extra > $OUT/b.json 2>&1 || { tail $OUT/b.json; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]);print('$args', d['roofline']['achieved'], d['roofline']['launch_ms'], d['config']['kernel'])"
done
