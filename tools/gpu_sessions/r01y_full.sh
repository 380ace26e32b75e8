set -u
cd $GRAFT_REPO_ROOT; OUT=$PWD/gpurun_out/r01y; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --config 5 --window 64 --steps 400 --warmup 5 --no-cpu-baseline > $OUT/c5_w64_k400.json 2>&1 || { tail $OUT/c5_w64_k400.json; exit 1; }
python -c "import json;d=json.loads(open('$OUT/c5_w64_k400.json').read().strip().splitlines()[-1]);print('c5 w64 k400', d['value'], d['ms_per_step'], d['roofline']['achieved'])"
timeout -k 10 200 python -u tools/sha_scale.py --chains 4096,16384,65536,131072,262144 > $OUT/sha_scale_auto.jsonl 2>&1 || { tail $OUT/sha_scale_auto.jsonl; exit 1; }
for a in "--gib 64 --hash gpu --window 32" "--gib 64 --hash gpu --window 64" "--gib 16 --hash host" "--gib 16 --k 32 --m 32 --hash gpu --window 32"; do
  timeout -k 10 300 python -u tools/e2e_bench.py $a > $OUT/e2e.json 2>&1 || { tail $OUT/e2e.json; exit 1; }
  echo "$a: $(tail -1 $OUT/e2e.json)"
done
