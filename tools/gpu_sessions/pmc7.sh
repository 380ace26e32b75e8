set -u
cd $GRAFT_REPO_ROOT; OUT=$PWD/gpurun_out/r01h; mkdir -p $OUT; export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/sq5 -o run -- python -u bench.py --config 5 --sweep=-1 --steps 2 --warmup 1 > $OUT/sq5.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_IFETCH SQ_IFETCH_LEVEL SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY --output-format csv -d $OUT/sqb5 -o run -- python -u bench.py --config 5 --sweep=-1 --steps 2 --warmup 1 > $OUT/sqb5.log 2>&1 || exit 1
echo done
