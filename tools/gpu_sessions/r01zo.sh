set -u
cd $GRAFT_REPO_ROOT; OUT=$PWD/gpurun_out/r01zo; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "ct_variants_identical or full_geometry_rs3232" -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --config 5 --sweep=-1,19,20,-1,19 --steps 60 --warmup 5 > $OUT/sweep.jsonl 2>$OUT/sweep.err || { tail $OUT/sweep.err; exit 1; }
cat $OUT/sweep.jsonl
