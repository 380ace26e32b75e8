set -u
cd $GRAFT_REPO_ROOT; OUT=$PWD/gpurun_out/r01zn; mkdir -p $OUT
export TMPDIR=/tmp
for v in -1 17; do
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/sq5_$v -o run -- python -u bench.py --config 5 --variant $v --sweep=$v --steps 2 --warmup 1 > $OUT/sq5_$v.log 2>&1 || { tail -5 $OUT/sq5_$v.log; exit 1; }
done
find $OUT -name "*counter_collection.csv"
