set -u
cd $GRAFT_REPO_ROOT; OUT=$PWD/gpurun_out/r01ze; mkdir -p $OUT
timeout -k 10 120 python -u tools/stress_rthx.py --runs 10 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2>$OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
