set -u
cd $GRAFT_REPO_ROOT; OUT=$PWD/gpurun_out/r01w; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_hashq.py tests/test_gpu_parity.py -k "hashq or shavs or window or geometry or edge_cases or segment_list or sha" -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for pf in 1 3; do
  timeout -k 10 200 python -u tools/sha_scale.py --pf $pf --chains 4096,16384,32768,65536,81920,98304,131072,196608,262144 > $OUT/scale_pf$pf.jsonl 2>&1 || { tail $OUT/scale_pf$pf.jsonl; exit 1; }
  grep chains $OUT/scale_pf$pf.jsonl
done
for hs in 0 1; do for w in 16 32 64; do
  timeout -k 10 200 python -u bench.py --config 5 --window $w --hash-stream $hs --steps 100 --warmup 5 --no-cpu-baseline > $OUT/c5_hs${hs}_w$w.json 2>&1 || { tail $OUT/c5_hs${hs}_w$w.json; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/c5_hs${hs}_w$w.json').read().strip().splitlines()[-1]);print('hs=$hs w=$w', d['value'], d['ms_per_step'], d['roofline']['achieved'])"
done; done
