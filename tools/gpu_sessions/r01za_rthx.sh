set -u
cd $GRAFT_REPO_ROOT; OUT=$PWD/gpurun_out/r01za; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "runtime_kernels or golden or per_segment or repair or degraded" -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for args in "--config 6" "--config 7" "--config 8" "--config 5 --generic"; do for rt in 0 2; do
  timeout -k 10 200 python -u bench.py $args --rt-mode $rt --steps 20 --warmup 3 --no-cpu-baseline --no-extra > $OUT/b.json 2>&1 || { tail $OUT/b.json; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]);print('$args rt=$rt', d['roofline']['achieved'], d['roofline']['launch_ms'])"
done; done
