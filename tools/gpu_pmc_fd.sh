#!/bin/bash
# SQ counters of the RS(32,32) rebuild kernels (config 6): where a wave's time goes in
# k_fftdec_m and k_rthx. One counter group per rocprofv3 run (kernel-trace only, no tracing).
# usage: tools/gpu_pmc_fd.sh <tag> "<erasures>:<fftdec-mode>:<fftdec-min> ..."
set -u
TAG=$1; CASES=$2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_ANY SQ_WAIT_INST_ANY"
G2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
for c in $CASES; do
  IFS=: read -r e mode fmin <<< "$c"
  for g in 1 2; do
    grp=G$g
    d="$OUT/e${e}_m${mode}_f${fmin}_g$g"
    timeout -s KILL 90 rocprofv3 --pmc ${!grp} --output-format csv -d "$d" -o run -- \
      python -u bench.py --config 6 --erasures "$e" --fftdec-mode "$mode" --fftdec-min "$fmin" \
      --no-cpu-baseline --no-extra --steps 5 --warmup 1 > "$d.log" 2>&1 \
      || { echo "pmc $c g$g failed rc=$?"; tail -5 "$d.log"; exit 1; }
    f=$(find "$d" -name "*counter_collection.csv" | head -1)
    cp "$f" "$OUT/pmc_e${e}_m${mode}_f${fmin}_g$g.csv"
  done
done
echo done
