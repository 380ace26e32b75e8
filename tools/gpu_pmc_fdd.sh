#!/bin/bash
# SQ counters of the formal-derivative decoder forms at 32 random erasures (config 6, decoder
# forced): k_fftdec_d (variant 70), k_fftdec_dp (-1), k_fftdec_dp with LDS DMA (71). One counter
# group per rocprofv3 run (kernel-trace only), plus a kernel-trace --stats run per form.
# usage: tools/gpu_pmc_fdd.sh <tag> "<variant> ..."
set -u
TAG=$1; VARS=${2:-"-1 70 71"}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_ANY SQ_WAIT_INST_ANY"
G2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
for v in $VARS; do
  d="$OUT/v${v}_stats"
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o run -- \
    python -u bench.py --config 6 --erasures 32 --fftdec-mode 2 --variant "$v" \
    --no-cpu-baseline --no-extra --steps 40 --warmup 30 > "$d.log" 2>&1 \
    || { echo "stats v$v failed rc=$?"; tail -5 "$d.log"; exit 1; }
  f=$(find "$d" -name "*kernel_stats.csv" | head -1)
  cp "$f" "$OUT/kernel_stats_v${v}.csv"
  for g in 1 2; do
    grp=G$g
    d="$OUT/v${v}_g$g"
    timeout -s KILL 90 rocprofv3 --pmc ${!grp} --output-format csv -d "$d" -o run -- \
      python -u bench.py --config 6 --erasures 32 --fftdec-mode 2 --variant "$v" \
      --no-cpu-baseline --no-extra --steps 5 --warmup 1 > "$d.log" 2>&1 \
      || { echo "pmc v$v g$g failed rc=$?"; tail -5 "$d.log"; exit 1; }
    f=$(find "$d" -name "*counter_collection.csv" | head -1)
    cp "$f" "$OUT/pmc_v${v}_g$g.csv"
  done
done
echo done
