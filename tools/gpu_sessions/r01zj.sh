set -u
cd $GRAFT_REPO_ROOT; OUT=$PWD/gpurun_out/r01zj; mkdir -p $OUT
for v in -1 12 -1 12 -1 12; do
  timeout -k 10 200 python -u bench.py --config 3 --variant $v --steps 200 --warmup 10 --no-cpu-baseline --no-extra > $OUT/b.json 2>$OUT/b.err || { tail $OUT/b.err; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]);print('config 3 variant $v', d['value'], d['roofline']['achieved'], d['roofline']['launch_ms'])" | tee -a $OUT/ab.txt
done
