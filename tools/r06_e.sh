#!/bin/bash
# default bench line (N = 1) with the new host_e2e legs
set -o pipefail
mkdir -p gpurun_out/r06e
timeout -k 10 400 python -u bench.py > gpurun_out/r06e/bench_default.json 2> gpurun_out/r06e/bench_default.err
rc=$?
tail -c 300 gpurun_out/r06e/bench_default.err
python - <<'P'
import json
d=json.loads(open("gpurun_out/r06e/bench_default.json").read().strip().splitlines()[-1])
print(json.dumps(d["extra"]["host_e2e"], indent=1))
print("value", d["value"], "frac", d["roofline"]["frac"])
P
exit $rc
