set -u
cd $GRAFT_REPO_ROOT; OUT=$PWD/gpurun_out/r01zg; mkdir -p $OUT
for g in 12 16 24; do
  echo -n "--gib $g gpu: " >> $OUT/e2e.txt
  timeout -k 10 200 python -u tools/e2e_bench.py --gib $g --hash gpu >> $OUT/e2e.txt 2>$OUT/e2e.err || { tail $OUT/e2e.err; exit 1; }
  echo -n "--gib $g host: " >> $OUT/e2e.txt
  timeout -k 10 200 python -u tools/e2e_bench.py --gib $g --hash host >> $OUT/e2e.txt 2>$OUT/e2e.err || { tail $OUT/e2e.err; exit 1; }
done
cat $OUT/e2e.txt
