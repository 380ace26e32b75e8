set -u
cd $GRAFT_REPO_ROOT; OUT=$PWD/gpurun_out/r01q; mkdir -p $OUT
for args in "--config 7 --rt-mode 0" "--config 7 --rt-mode 1" "--config 8 --rt-mode 0" "--config 8 --rt-mode 1" "--config 6 --rt-mode 0" "--config 6 --rt-mode 1"; do
  timeout -k 10 200 python -u bench.py $args --steps 10 --warmup 2 --no-cpu-baseline --no-extra > $OUT/b.json 2>&1 || { tail $OUT/b.json; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]);print('$args', d['roofline']['achieved'], d['roofline']['launch_ms'], d['config']['kernel'])"
done
