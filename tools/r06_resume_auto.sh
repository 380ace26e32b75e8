#!/bin/bash
# Resume on by itself below 12 host threads: the pipeline tests first, then records_bench's
# four-file stream (pieces source) with the knob unset (auto) and forced off, 8 and 4 threads,
# alternating twice; 16 threads unset (auto = off) once as the default's check.
set -o pipefail
OUT=gpurun_out/r06resauto; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_pipeline.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
run() {  # name threads [env value]
  if [ -n "${3:-}" ]; then export CEC_PIPELINE_RESUME=$3; else unset CEC_PIPELINE_RESUME; fi
  CEC_PIPELINE_TRACE=1 timeout -k 10 200 python -u tools/records_bench.py --gib 8 --modes hybrid --reps 1 --stream 4 --pieces --threads $2 > $OUT/rb_$1.jsonl 2>&1 || exit 1
  echo "== $1"; grep -h "records_stream" $OUT/rb_$1.jsonl | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d.get('GBps'), d.get('cpu_seconds'), d.get('file_done_s'))"
  grep "cec_pipeline" $OUT/rb_$1.jsonl | tail -1 | grep -o "resume [01]"
}
for rep in 1 2; do
  for th in 8 4; do
    run auto_${th}_$rep $th
    run off_${th}_$rep $th 0
  done
done
run auto_16 16
