set -u
cd $GRAFT_REPO_ROOT; OUT=$PWD/gpurun_out/r01d; mkdir -p $OUT; export TMPDIR=/tmp
for v in 0 3; do
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/sq5_$v -o run -- python -u bench.py --config 5 --variant $v --sweep=$v --steps 2 --warmup 1 > $OUT/sq5_$v.log 2>&1 || exit 1
done
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/sq2 -o run -- python -u bench.py --config 2 --sweep=-1 --steps 2 --warmup 1 > $OUT/sq2.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_IFETCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_LDS SQ_IFETCH_LEVEL --output-format csv -d $OUT/sqb5 -o run -- python -u bench.py --config 5 --variant 3 --sweep=3 --steps 2 --warmup 1 > $OUT/sqb5.log 2>&1 || echo "sqb5 failed"
echo done
