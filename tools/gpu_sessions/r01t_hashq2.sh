set -u
cd $GRAFT_REPO_ROOT; OUT=$PWD/gpurun_out/r01t; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_hashq.py tests/test_gpu_parity.py -k "hashq or shavs or window or geometry or edge_cases or segment_list or sha" -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for w in 16 32; do
  timeout -k 10 200 python -u bench.py --config 5 --window $w --steps 100 --warmup 5 --no-cpu-baseline > $OUT/c5_w$w.json 2>&1 || { tail $OUT/c5_w$w.json; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/c5_w$w.json').read().strip().splitlines()[-1]);print('w=$w', d['value'], d['ms_per_step'], d['roofline']['achieved'])"
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o c5 -- python -u bench.py --config 5 --window 16 --steps 100 --warmup 5 --no-cpu-baseline > $OUT/rocprof_c5.log 2>&1 || { tail $OUT/rocprof_c5.log; exit 1; }
find $OUT/prof -name "*kernel_stats*" -exec cp {} $OUT/ \;
for h in gpu host; do
  timeout -k 10 300 python -u tools/e2e_bench.py --gib 16 --hash $h --window 32 > $OUT/e2e_$h.json 2>&1 || { tail $OUT/e2e_$h.json; exit 1; }
  tail -1 $OUT/e2e_$h.json
done
