set -u
cd $GRAFT_REPO_ROOT; OUT=$PWD/gpurun_out/r01u; mkdir -p $OUT
timeout -k 10 200 python -u -m pytest tests/test_gpu_hashq.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for pf in 1 2; do
  timeout -k 10 200 python -u tools/sha_scale.py --pf $pf > $OUT/scale_pf$pf.jsonl 2>&1 || { tail $OUT/scale_pf$pf.jsonl; exit 1; }
  cat $OUT/scale_pf$pf.jsonl | grep chains
done
timeout -k 10 200 python -u tools/sha_scale.py --pf 1 --stride 16384 > $OUT/scale_dense.jsonl 2>&1 || { tail $OUT/scale_dense.jsonl; exit 1; }
grep chains $OUT/scale_dense.jsonl
for pf in 1 2; do
  timeout -k 10 200 python -u bench.py --config 5 --window 16 --tick-pf $pf --steps 100 --warmup 5 --no-cpu-baseline > $OUT/c5_pf$pf.json 2>&1 || { tail $OUT/c5_pf$pf.json; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/c5_pf$pf.json').read().strip().splitlines()[-1]);print('pf=$pf', d['value'], d['ms_per_step'], d['roofline']['achieved'])"
done
