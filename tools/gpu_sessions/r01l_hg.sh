set -u
cd $GRAFT_REPO_ROOT; OUT=$PWD/gpurun_out/r01l; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "variants or rs3232" -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --config 5 --sweep=-1,10,11,12,13,14,15,16 --steps 20 --warmup 3 > $OUT/sweep5.jsonl 2>&1 || { tail $OUT/sweep5.jsonl; exit 1; }
cat $OUT/sweep5.jsonl
